// ORB extraction on gfx950 — SURVEY.md §8a rows E1-E7.
//
// Replaces ORB_SLAM::ORBextractor (src/ORBextractor.cc:464-998) for a batch
// of independent frames. Pipeline per batch (all kernels batched over frames,
// one HIP stream, no host round trip):
//
//   k_resize  x (nlevels-1)  level l from level l-1 (cv::resize INTER_LINEAR,
//                            11-bit fixed point; ComputePyramid :922-998)
//   k_blur_fast              one 64x64 tile per workgroup: 7x7 sigma-2
//                            Gaussian of every level (:842) and, from the same
//                            LDS tile, the FAST-9 score map of the level
//   k_fast_cells             one workgroup per (frame, grid cell): corners of
//                            the cell window from the score map, in-cell NMS,
//                            threshold fallback 20 -> 7, row-major compaction
//                            (ComputeKeyPoints :575-689)
//   k_select                 one workgroup per (frame, level): quota
//                            redistribution (:695-721) + retainBest per cell
//                            and per level (:734-752)
//   k_describe               one wave per keypoint: IC_Angle (:131-158) on
//                            the unblurred level, rBRIEF (:162-201) on the
//                            blurred level, scale to level 0 (:865-871)
//
// Levels are stored without the 16-px border frame: every border read the
// reference makes is reflect-101 of the level interior, so it is addressed on
// the fly (reflect101) instead of materialised.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

#include "common.h"
#include "libm_sincosf.h"
#include "orb_pattern.h"
#include "select.h"

#define GF_MAX_LEVELS 12

namespace {

__constant__ uint32_t c_pattern8[256];  // test i: (x0, y0, x1, y1) of its two points as int8
// IC_Angle row weights by |v| (k_describe): [16][8] dwords of bytes u + 15 for
// |u| <= umax[|v|] (else 0), then [16][8] dwords of the 0/1 patch mask (column
// c = 4 j + b is u = c - 15; column 31 weighs 0)
__constant__ uint32_t c_ic_tab[256];

struct LevelGeom {
    int nlevels;
    int w[GF_MAX_LEVELS], h[GF_MAX_LEVELS];
    int pw[GF_MAX_LEVELS];          // row pitch of the blurred / score planes (64-B multiple)
    long long off[GF_MAX_LEVELS];   // pyramid slab offset (levels >= 1)
    long long boff[GF_MAX_LEVELS];  // blurred slab offset (all levels)
    long long slab, bslab;          // bytes per frame
    float scale[GF_MAX_LEVELS];
    // cells
    int cell_begin[GF_MAX_LEVELS + 1];
    int ncells;
    int nfcell[GF_MAX_LEVELS], ndesired[GF_MAX_LEVELS];
    long long lvl_off[GF_MAX_LEVELS + 1];  // level list offsets (entries)
    // blur tiling
    int tile_begin[GF_MAX_LEVELS + 1];
    int tiles_x[GF_MAX_LEVELS];
};

struct CellInfo {
    int level, x0, y0, w, h, valid;
    long long cap_off;
    int cap;
    int band;  // 0: the window fits k_fast_cells' LDS; else rows per band of k_fast_cells_band
};

struct Planes {
    const uint8_t* img0;
    long long fstride0;
    int stride0;
    const uint8_t* const* ptrs;  // optional: level 0 of frame f at ptrs[f] (device pointer table)
    uint8_t* pyr;
    uint8_t* blur;
};

__device__ __forceinline__ const uint8_t* level_plane(const Planes& P, const LevelGeom& g, int f, int l,
                                                      int& stride) {
    if (l == 0) {
        stride = P.stride0;
        return P.ptrs ? P.ptrs[f] : P.img0 + (long long)f * P.fstride0;
    }
    stride = g.pw[l];  // levels >= 1: rows pitched to 64 B like the blurred planes
    return P.pyr + (long long)f * g.slab + g.off[l];
}

// Keypoint list entries of the cell and level lists.
// FAST_SCORE (1): u32 score << 24 | y << 12 | x, the score the FAST map holds.
// HARRIS_SCORE (0): u64 key << 32 | y << 12 | x, key = HarrisResponses' float
// response (ORBextractor.cc:86-127, 667-670) as an order-preserving int32, so
// retainBest's float comparisons (KeypointResponseGreater) are key comparisons.
template <typename E>
struct Ent;
template <>
struct Ent<uint32_t> {
    __host__ __device__ static int key(uint32_t e) { return (int)(e >> 24); }
    __device__ static float response(uint32_t e) { return (float)(e >> 24); }
};
template <>
struct Ent<uint64_t> {
    __host__ __device__ static int key(uint64_t e) { return (int)(uint32_t)(e >> 32); }
    __device__ static float response(uint64_t e) {
        const int k = key(e);
        return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff);
    }
};
template <typename E>
struct EntGreater {  // KeypointResponseGreater on list entries
    __host__ __device__ bool operator()(E a, E b) const { return Ent<E>::key(a) > Ent<E>::key(b); }
};
__device__ __forceinline__ int float_key(float v) {
    int b = __float_as_int(v);
    if (b == (int)0x80000000) b = 0;  // -0 == +0
    return b >= 0 ? b : b ^ 0x7fffffff;
}

// HarrisResponses(cellImage, kps, blockSize 7, HARRIS_K 0.04) for one
// keypoint at level pixel (cx, cy) (ORBextractor.cc:86-127): integer
// gradient moments over the 7x7 block, then the reference's float expression
// in its evaluation order (no contraction: -ffp-contract=off).
__device__ float harris_response(const uint8_t* Pl, int step, int cx, int cy) {
    const uint8_t* ptr0 = Pl + (long long)(cy - 3) * step + (cx - 3);
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < 7; i++) {
        const uint8_t* p = ptr0 + (long long)i * step;
#pragma unroll
        for (int j = 0; j < 7; j++, p++) {
            const int Ix = (p[1] - p[-1]) * 2 + (p[-step + 1] - p[-step - 1]) + (p[step + 1] - p[step - 1]);
            const int Iy = (p[step] - p[-step]) * 2 + (p[step - 1] - p[-step - 1]) + (p[step + 1] - p[-step + 1]);
            a += Ix * Ix;
            b += Iy * Iy;
            c += Ix * Iy;
        }
    }
    float scale = (1 << 2) * 7 * 255.0f;
    scale = 1.0f / scale;
    const float scale_sq_sq = scale * scale * scale * scale;
    const float harris_k = 0.04f;
    return ((float)a * b - (float)c * c - harris_k * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
}

// The list entry of a corner at level pixel (X, Y) with FAST score S.
template <typename E>
__device__ __forceinline__ E cell_entry(int S, int X, int Y, const Planes& P, const LevelGeom& g, int f, int l) {
    if constexpr (sizeof(E) == 4) {
        return ((uint32_t)S << 24) | ((uint32_t)Y << 12) | (uint32_t)X;
    } else {
        int step;
        const uint8_t* Pl = level_plane(P, g, f, l, step);
        return ((uint64_t)(uint32_t)float_key(harris_response(Pl, step, X, Y)) << 32) | ((uint64_t)Y << 12) |
               (uint64_t)X;
    }
}

// -------------------------------------------------------------- k_pyramid
// cv::resize INTER_LINEAR, level l from level l-1 (ORBextractor.cc:1063-1068),
// every level in one launch. xtab[dx] = (sx, a0 | a1<<16), ytab[dy] = (sy,
// b0 | b1<<16) are OpenCV's fixed-point coefficients (2048 = 1.0), made on the
// host with its float arithmetic.
// Each level is cut into the same nbx x nby grid of blocks (block k of a
// level of width w owns columns k w / nbx .. (k + 1) w / nbx - 1). One
// 256-thread workgroup per (frame, block) takes the level-0 pixels its block
// column needs through all the levels into LDS once, then makes level 1, 2,
// ... from the previous level in LDS: at each level the pixels it owns plus
// the few the next level's owned pixels read beyond them (the required span,
// PyrSpan.lo .. hi, made on the host from the tables top-down). A pixel is a
// function of the level below only, so a span pixel recomputed by a
// neighbouring block is the same byte; only the owner stores it. No
// workgroup waits for another, and one launch replaces one per level.
struct PyrSpan {
    int16_t lo, hi;    // required pixels of the level, inclusive
    int16_t olo, ohi;  // owned pixels [olo, ohi) (level 0: none)
};
struct PyrGeom {
    int nbx, nby;
    int rx, ry;     // dwords per block-column / block-row record
    int lds_a;      // bytes of the even levels' buffer (the odd levels' follows)
    int lds_img;    // bytes of both buffers (the records follow)
};
#define PYR_NT 512  // threads per block
#define PYR_G 4     // output pixels per item (a row's 4 consecutive columns)

__device__ __forceinline__ int pyr_pitch(int span) { return (span + 8 + 3) & ~3; }

// floor(i / n) for 0 <= i < 2^20, n >= 1, rn = 1 / n in float: the product's
// relative error (~2^-22) stays below the 0.5 / n margin the + 0.5 leaves
// while i < 2^21
__device__ __forceinline__ int pyr_div(int i, float rn) { return (int)(((float)i + 0.5f) * rn); }

// Records, made on the host, staged in LDS with the level-0 pixels (the level
// passes then wait on LDS only). Block column: the PyrSpan of each of the nl
// levels (2 dwords), then per level 1 .. nl-1 and column group (G columns
// from x0 = lo + G g): {c0 | d1 << 16 | d2 << 20 | d3 << 24 | own << 28} and
// the G weights a0 | a1 << 16; c0 = the first column's left tap in the
// source span, d_k = column k's left tap past c0, own = the columns this
// block stores. Block row: spans, then per level and row {r0 | r1 << 16 |
// own << 31} (source rows in the source span, clamped as OpenCV clamps) and
// b0 | b1 << 16.
// A level pass: thread t takes column group g = t % ng in rows t / ng,
// + NT / ng, ... Per source row: the three LDS dwords from the group's first
// tap realigned to two (v_alignbyte), each column's tap pair picked as 16-bit
// lanes (v_perm_b32) and weighted by v_dot2_u32_u16 (p0 a0 + p1 a1, the
// exact sum); then OpenCV's vertical step ((b0 (t0 >> 4)) >> 16) +
// ((b1 (t1 >> 4)) >> 16) + 2 >> 2, at most 255 as the weights sum to at most
// 2049 (checked on the host), so no clamp. The host takes G = 4 when every
// group's taps lie within 8 bytes of its first (scale <= 2), else G = 1.
template <int G>
__global__ __launch_bounds__(PYR_NT) void k_pyramid(Planes P, LevelGeom g, PyrGeom pg,
                                                    const uint32_t* __restrict__ xrec,
                                                    const uint32_t* __restrict__ yrec) {
    gfd::ext_prio();
    extern __shared__ __align__(16) uint8_t pyr_lds[];
    int blk, f;
    gfd::xcd_block(blk, f);
    const int tid = threadIdx.x;
    const int kx = blk % pg.nbx, ky = blk / pg.nbx;
    const int nl = g.nlevels;
    uint32_t* tx = reinterpret_cast<uint32_t*>(pyr_lds + pg.lds_img);
    uint32_t* ty = tx + pg.rx;
    for (int i = tid; i < pg.rx; i += PYR_NT) tx[i] = gfd::ldg(xrec + (long long)kx * pg.rx + i);
    for (int i = tid; i < pg.ry; i += PYR_NT) ty[i] = gfd::ldg(yrec + (long long)ky * pg.ry + i);
    auto span = [](const uint32_t* r, int l) {
        return __builtin_bit_cast(PyrSpan, make_uint2(r[2 * l], r[2 * l + 1]));
    };
    {  // level 0: the block's source rectangle, realigned so LDS column 0 is its first column
        const uint32_t* gx = xrec + (long long)kx * pg.rx;
        const uint32_t* gy = yrec + (long long)ky * pg.ry;
        const PyrSpan sx = __builtin_bit_cast(PyrSpan, make_uint2(gfd::ldg(gx), gfd::ldg(gx + 1)));
        const PyrSpan sy = __builtin_bit_cast(PyrSpan, make_uint2(gfd::ldg(gy), gfd::ldg(gy + 1)));
        const int w0 = sx.hi - sx.lo + 1, nr = sy.hi - sy.lo + 1, pitch = pyr_pitch(w0), ndw = pitch >> 2;
        const float rn = 1.0f / (float)ndw;
        int stride;
        const uint8_t* S = level_plane(P, g, f, 0, stride) + sx.lo;
        uint32_t* A = reinterpret_cast<uint32_t*>(pyr_lds);
        constexpr int LB = 8;  // dwords per thread per batch, all in flight
        if ((stride & 3) == 0 && ndw <= PYR_NT) {
            // rows share one byte shift: thread t owns dword column t % ndw of
            // rows t / ndw + k rstep, one multiply-add from row to row
            const int q = tid % ndw, r0 = tid / ndw, rstep = PYR_NT / ndw;
            // (a column past the span loads the span's last dword and stores 0)
            const uintptr_t a0 = (uintptr_t)(S + sy.lo * stride) + 4 * min(q, (w0 - 1) >> 2);
            const uint32_t sh = (uint32_t)(a0 & 3);
            const bool col = r0 < rstep && 4 * q < w0, two = col && sh != 0 && 4 * q + 4 - (int)sh < w0;
            const uint32_t* c0 = reinterpret_cast<const uint32_t*>(a0 & ~(uintptr_t)3);
            const int s4 = stride >> 2;
            for (int rb = r0; rb < nr; rb += LB * rstep) {
                uint32_t lo[LB], hi[LB];
#pragma unroll
                for (int k = 0; k < LB; k++) {  // unconditional loads at clamped rows
                    const uint32_t* p = c0 + (long long)min(rb + k * rstep, nr - 1) * s4;
                    lo[k] = gfd::ldg(p);
                    hi[k] = gfd::ldg(p + (two ? 1 : 0));
                }
#pragma unroll
                for (int k = 0; k < LB; k++) {
                    const int r = rb + k * rstep;
                    if (r0 < rstep && r < nr) A[r * ndw + q] = col ? __builtin_amdgcn_alignbyte(hi[k], lo[k], sh) : 0u;
                }
            }
        } else
        for (int i0 = 0; i0 < nr * ndw; i0 += PYR_NT * LB) {
            uint32_t lo[LB], hi[LB], sh[LB];
#pragma unroll
            for (int k = 0; k < LB; k++) {
                const int i = i0 + PYR_NT * k + tid;
                const int r = pyr_div(i, rn), q = i - r * ndw;
                lo[k] = hi[k] = sh[k] = 0u;
                if (r < nr && 4 * q < w0) {
                    const uintptr_t a = (uintptr_t)(S + (sy.lo + r) * stride) + 4 * q;
                    const uintptr_t al = a & ~(uintptr_t)3;
                    sh[k] = (uint32_t)(a & 3);
                    // the second aligned dword only when one of the needed bytes lies in it
                    const bool two = sh[k] != 0 && 4 * q + 4 - (int)sh[k] < w0;
                    lo[k] = gfd::ldg(reinterpret_cast<const uint32_t*>(al));
                    hi[k] = gfd::ldg(reinterpret_cast<const uint32_t*>(two ? al + 4 : al));
                }
            }
#pragma unroll
            for (int k = 0; k < LB; k++) {
                const int i = i0 + PYR_NT * k + tid;
                if (i < nr * ndw) A[i] = __builtin_amdgcn_alignbyte(hi[k], lo[k], sh[k]);
            }
        }
    }
    __syncthreads();
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    int offx = 2 * nl, offy = 2 * nl;  // the level's first group / row entry in the records
    for (int l = 1; l < nl; l++) {
        const PyrSpan ssx = span(tx, l - 1), dsx = span(tx, l), dsy = span(ty, l);
        const uint32_t srcb = (l - 1) & 1 ? pg.lds_a : 0u, dstb = l & 1 ? pg.lds_a : 0u;
        const int sp = pyr_pitch(ssx.hi - ssx.lo + 1);
        const int dspan = dsx.hi - dsx.lo + 1, dp = pyr_pitch(dspan), nrow = dsy.hi - dsy.lo + 1;
        const int ng = (dspan + G - 1) / G, rstep = PYR_NT / ng;
        const int r00 = pyr_div(tid, 1.0f / (float)ng), gi = tid - r00 * ng;
        const int dw = g.pw[l];
        const int x0 = dsx.lo + G * gi;
        uint8_t* D = P.pyr + (long long)f * g.slab + g.off[l] + x0;
        uint32_t sel[G], wgt[G], own = 0, cq = 0, csh = 0;
        if (r00 < rstep) {
            const uint32_t* gr = tx + offx + (1 + G) * gi;
            const uint32_t h = gr[0];
            own = h >> 28;
            cq = (h & 0xffffu) >> 2;
            csh = h & 3u;
#pragma unroll
            for (int k = 0; k < G; k++) {
                const uint32_t d = k == 0 ? 0u : (h >> (12 + 4 * k)) & 15u;
                sel[k] = d * 0x00010001u + 0x0c010c00u;  // bytes d, d + 1 as 16-bit lanes
                wgt[k] = gr[1 + k];
            }
        }
        const uint32_t* rows = ty + offy;
        for (int r = r00; r < nrow && r00 < rstep; r += rstep) {
            const uint32_t rr = rows[2 * r], bb = rows[2 * r + 1];
            const uint32_t* s0 = reinterpret_cast<const uint32_t*>(pyr_lds + srcb + (rr & 0x7fffu) * sp) + cq;
            const uint32_t* s1 = reinterpret_cast<const uint32_t*>(pyr_lds + srcb + ((rr >> 16) & 0x7fffu) * sp) + cq;
            const uint32_t u0 = s0[0], u1 = s0[1], u2 = s0[2], v0 = s1[0], v1 = s1[1], v2 = s1[2];
            const uint32_t ua = __builtin_amdgcn_alignbyte(u1, u0, csh), ub = __builtin_amdgcn_alignbyte(u2, u1, csh);
            const uint32_t va = __builtin_amdgcn_alignbyte(v1, v0, csh), vb = __builtin_amdgcn_alignbyte(v2, v1, csh);
            const uint32_t b0 = bb & 0xffffu, b1 = bb >> 16;
            uint32_t o = 0;
#pragma unroll
            for (int k = 0; k < G; k++) {
                const u16x2 w = __builtin_bit_cast(u16x2, wgt[k]);
                const uint32_t t0 =
                    __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(ub, ua, sel[k])), w, 0u, false);
                const uint32_t t1 =
                    __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(vb, va, sel[k])), w, 0u, false);
                const uint32_t v = ((__mul24(b0, t0 >> 4) >> 16) + (__mul24(b1, t1 >> 4) >> 16) + 2) >> 2;
                o |= v << (8 * k);
            }
            if constexpr (G == 4) {
                *reinterpret_cast<uint32_t*>(pyr_lds + dstb + r * dp + G * gi) = o;
            } else {
#pragma unroll
                for (int k = 0; k < G; k++) pyr_lds[dstb + r * dp + G * gi + k] = (uint8_t)(o >> (8 * k));
            }
            if ((rr >> 31) && own) {
                uint8_t* q = D + (dsy.lo + r) * dw;
                if (G == 4 && own == 0xfu) {  // column groups start at multiples of 4 (host plan): one dword
                    *reinterpret_cast<uint32_t*>(q) = o;
                } else if (own == (1u << G) - 1u) {
#pragma unroll
                    for (int k = 0; k < G; k++) q[k] = (uint8_t)(o >> (8 * k));
                } else {
#pragma unroll
                    for (int k = 0; k < G; k++)
                        if ((own >> k) & 1u) q[k] = (uint8_t)(o >> (8 * k));
                }
            }
        }
        offx += (1 + G) * ng;
        offy += 2 * nrow;
        __syncthreads();
    }
}

// -------------------------------------------------------------- FAST-9
__device__ __forceinline__ void circle_vals(const uint8_t* roi, int rw, int px, int py, int c[16]) {
    const uint8_t* p = roi + py * rw + px;
    c[0] = p[3 * rw];
    c[1] = p[3 * rw + 1];
    c[2] = p[2 * rw + 2];
    c[3] = p[rw + 3];
    c[4] = p[3];
    c[5] = p[-rw + 3];
    c[6] = p[-2 * rw + 2];
    c[7] = p[-3 * rw + 1];
    c[8] = p[-3 * rw];
    c[9] = p[-3 * rw - 1];
    c[10] = p[-2 * rw - 2];
    c[11] = p[-rw - 3];
    c[12] = p[-3];
    c[13] = p[rw - 3];
    c[14] = p[2 * rw - 2];
    c[15] = p[3 * rw - 1];
}

// FAST-9 segment test and OpenCV cornerScore<16> in closed form, branch-free
// on packed 16-bit pairs. With d_k = v - c_k, cornerScore returns
// max(th, D, B) - 1 where D = max over the 16 arcs of 9 of min_arc d and
// B = max over arcs of min_arc (-d) (its early-outs only skip arcs that cannot
// raise the maximum), and the segment test at th passes exactly when
// max(D, B) > th. So M = max(D, B) gives both: corner iff M > th, score
// M - 1. (d, -d) share one register. The arcs starting at 2i and 2i + 1 share
// the 8 values 2i + 1 .. 2i + 8, built by doubling over odd starts only
// (8 + 8 + 8 v_pk_min_i16), then each pair of arcs costs 2 mins and 2 maxes.
typedef short gf_s2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int fast_max_arc(int v, const int c[16]) {
    const gf_s2 vn = {(short)v, (short)-v}, sgn = {-1, 1};
    gf_s2 p[16], m2[8], m4[8], m8[8];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const gf_s2 cc = {(short)c[k], (short)c[k]};
        p[k] = cc * sgn + vn;  // (v - c, c - v): one v_pk_mad_i16
    }
#pragma unroll
    for (int i = 0; i < 8; i++) m2[i] = __builtin_elementwise_min(p[2 * i + 1], p[(2 * i + 2) & 15]);
#pragma unroll
    for (int i = 0; i < 8; i++) m4[i] = __builtin_elementwise_min(m2[i], m2[(i + 1) & 7]);
#pragma unroll
    for (int i = 0; i < 8; i++) m8[i] = __builtin_elementwise_min(m4[i], m4[(i + 2) & 7]);
    gf_s2 mx = __builtin_elementwise_min(p[0], m8[0]);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        if (i) mx = __builtin_elementwise_max(mx, __builtin_elementwise_min(p[2 * i], m8[i]));
        mx = __builtin_elementwise_max(mx, __builtin_elementwise_min(m8[i], p[(2 * i + 9) & 15]));
    }
    return max((int)mx.x, (int)mx.y);
}

// Exclusive scan of one int per thread across one wave (total: the wave's sum).
__device__ __forceinline__ int wave_scan_excl(int v, int& total) {
    const int lane = threadIdx.x & 63;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

// Exclusive scan of one int per thread across a 256-thread workgroup.
__device__ int block_scan_256(int v, int* tmp, int& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    int base = 0;
    for (int i = 0; i < wid; i++) base += tmp[i];
    total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
    __syncthreads();
    return base + x - v;
}

// -------------------------------------------------------------- k_blur_fast
// One 64 x BT_H (64) tile of one level per 256-thread workgroup, its 3-px halo staged
// in LDS once and used twice:
//   * GaussianBlur 7x7 sigma 2 (reflect-101 border; ORBextractor.cc:842):
//     integer row pass, column pass with the (s + 2^15) >> 16 cast;
//   * the FAST-9 score map of the unblurred level at iniThFAST (:621):
//     S + 1 (S = cornerScore<16> <= 254) for a pixel that passes the segment
//     test, else 0 (and 0 within 3 px of the level border). The cells run
//     their fast_th pass, NMS included, from this map; the rare cell that
//     retries at minThFAST (:623-628) recomputes its window from the level
//     (k_fast_cells).
// LDS column j of the source tile holds x = X0 - 4 + j, so the tile's rows are
// whole dwords, loaded as aligned global dwords realigned with v_alignbyte
// (two loads per dword, all in flight together); only the dwords at the
// level's left and right edges load bytes through reflect-101. The row pass makes four outputs from
// three LDS dwords with v_dot4_u32_u8 (two per output: the 7 taps are bytes).
// Two rows' sums share a dword (each is at most 257 * 255 = 65535). Thread t
// then owns the pixel quad x = X0 + 4 (t & 15) .. +3 in rows 2 (t >> 4) and
// +1: four ds_read_b128 of row-pair sums, four v_dot2_u32_u16 per pixel for
// the column pass (the taps sum to 257, so the rounded value saturates at 255
// as saturate_cast does), one dword store per quad and row for the blurred plane, and the
// 4-point compass pre-test on the quad at once in packed 16-bit lanes (bytes
// 0/2 and 1/3 of the dword; the sign of c + th - v is "darker", of
// v + th - c "brighter"). The few pixels that pass are compacted into an LDS
// list (one workgroup scan), the full segment test + cornerScore runs on
// that list so whole waves do it, the scores land in an LDS score tile and go
// out as one dword per quad and row. The planes are pitched to 64 B, so a
// quad past the level's right edge writes the row padding.
#define BT_W 64
// BT_SKIP_PAST: waves of a tile's column / compass pass skip rows past the level
#ifndef BT_SKIP_PAST
#define BT_SKIP_PAST 1
#endif
#ifndef BT_H
#define BT_H 64
#endif
#define BT_R (BT_H + 6)   // source rows
#define BT_SW (BT_W + 8)  // source row: 72 bytes = 18 dwords, x = X0 - 4 .. X0 + 67
// LDS pitch of a source row: 24 dwords, so rows two apart (the two 16-lane
// halves of a ds_read_b32 group in the row and compass passes) sit 16 banks
// apart (mod 32): conflict-free, where the 18-dword pitch made them 2-way
#define BT_SP 96
#define BT_NQ (BT_H / 32) // row blocks of 32 per thread (quad x 2 rows each)
#define BT_U32 ((BT_R / 2) * BT_W > BT_W * BT_H / 2 ? (BT_R / 2) * BT_W : BT_W * BT_H / 2)

typedef short gf_i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ gf_i16x2 as_i16x2(uint32_t v) { return __builtin_bit_cast(gf_i16x2, v); }
__device__ __forceinline__ uint32_t as_u32(gf_i16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// Compass pre-test of FAST-9 on two pixels packed as 16-bit lanes (values
// 0..255): a 9-arc of the 16-ring covers two neighbouring compass points
// (ring positions 0, 4, 8, 12), both darker or both brighter than v by more
// than th. Returns the lanes' sign bits (bit 15: lane 0, bit 31: lane 1).
__device__ __forceinline__ uint32_t compass2(uint32_t v, uint32_t c0, uint32_t c4, uint32_t c8, uint32_t c12,
                                             uint32_t th2) {
    const gf_i16x2 V = as_i16x2(v), T = as_i16x2(th2), VT = V + T;
    const uint32_t d0 = as_u32(as_i16x2(c0) + T - V), d4 = as_u32(as_i16x2(c4) + T - V);
    const uint32_t d8 = as_u32(as_i16x2(c8) + T - V), d12 = as_u32(as_i16x2(c12) + T - V);
    const uint32_t b0 = as_u32(VT - as_i16x2(c0)), b4 = as_u32(VT - as_i16x2(c4));
    const uint32_t b8 = as_u32(VT - as_i16x2(c8)), b12 = as_u32(VT - as_i16x2(c12));
    return (((d0 | d8) & (d4 | d12)) | ((b0 | b8) & (b4 | b12))) & 0x80008000u;
}

__device__ __forceinline__ uint32_t bytes02(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c020c00u); }
__device__ __forceinline__ uint32_t bytes13(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c030c01u); }

__global__ __launch_bounds__(256) void k_blur_fast(Planes P, LevelGeom g, uint8_t* __restrict__ score, int map_th) {
    gfd::ext_prio();
    __shared__ __align__(16) uint8_t src[BT_R][BT_SP];
    // the row sums (rows 2p | 2p+1 << 16) are dead once the column pass has
    // read them; the candidate list, written after the scan's barriers, reuses them
    __shared__ __align__(16) uint32_t u32buf[BT_U32];
    __shared__ __align__(16) uint32_t sco[BT_H][BT_W / 4];
    __shared__ int scan_tmp[4];
    uint32_t(*rows2)[BT_W] = reinterpret_cast<uint32_t(*)[BT_W]>(u32buf);
    uint16_t* cand = reinterpret_cast<uint16_t*>(u32buf);
    int t, f;
    gfd::xcd_block(t, f);
    const int tid = threadIdx.x;
    int l = 0;
#pragma unroll
    for (int i = 1; i < GF_MAX_LEVELS; i++) l += (i < g.nlevels && t >= g.tile_begin[i]) ? 1 : 0;
    t -= g.tile_begin[l];
    const int tx = t % g.tiles_x[l], ty = t / g.tiles_x[l];
    const int w = g.w[l], h = g.h[l], pw = g.pw[l];
    const int X0 = tx * BT_W, Y0 = ty * BT_H;
    int stride;
    const uint8_t* S = level_plane(P, g, f, l, stride);
    {
        // BT_R rows x 18 dwords. Thread (lr, lq) = (tid / 18, tid % 18) owns
        // dword column lq of rows lr, lr + 14, ... (252 threads, 14 rows a
        // sweep), so its x range and LDS column are fixed. Rows reflect-101 at
        // the top and bottom (a uniform test per tile); in a level-0 image
        // whose rows are not dword-aligned the byte shift varies by row.
        constexpr int NQD = BT_SW / 4, LR = 256 / NQD, NI = (BT_R + LR - 1) / LR;
        const int lr = tid / NQD, lq = tid - lr * NQD;
        const int x0 = X0 - 4 + 4 * lq;
        const bool yin = Y0 >= 3 && Y0 + BT_R - 3 <= h;
        // Every lane loads the two aligned dwords holding its four source bytes
        // and picks them with one v_perm_b32: inside the row the bytes are
        // consecutive (the selector is the address's byte shift), at the x
        // borders they are reflect-101 positions, which span at most 4 bytes
        // (selector offsets <= 6 from the aligned base). No branch, so all the
        // stage's loads are in flight together. An aligned dword holding a
        // byte of the row never crosses a page; the second dword is taken
        // only when a byte lies in it.
        uint32_t lo[NI], hi[NI], sel[NI];
        int pj[4];
#pragma unroll
        for (int j = 0; j < 4; j++) pj[j] = gfd::reflect101(min(x0 + j, w + 2), w);
        const int pmin = min(min(pj[0], pj[1]), min(pj[2], pj[3]));
        if (((uintptr_t)S & 3u) == 0 && (stride & 3) == 0) {
            // dword-aligned rows (the pitched levels >= 1; level 0 when its
            // rows are): the byte offsets, the selector and the second dword
            // are the same in every row, only the row address changes
            const int pb = pmin & ~3;
            const int o0 = pj[0] - pb, o1 = pj[1] - pb, o2 = pj[2] - pb, o3 = pj[3] - pb;
            const bool two = max(max(o0, o1), max(o2, o3)) >= 4;
            const uint32_t sl = (uint32_t)o0 | (uint32_t)o1 << 8 | (uint32_t)o2 << 16 | (uint32_t)o3 << 24;
            static_assert(LR * (NI - 1) + LR - 1 < BT_R, "every row of a sweep exists");
            if (yin) {
                // interior rows (most tiles): the lane's rows lr + LR k are one
                // multiply-add from its first row, no reflect per row
                const uint8_t* row0 = S + (long long)(Y0 + lr - 3) * stride + pb;
                const long long sweep = (long long)LR * stride;
#pragma unroll
                for (int k = 0; k < NI; k++) {
                    sel[k] = sl;
                    lo[k] = hi[k] = 0u;
                    if (lr < LR) {  // both loads unconditional (the second re-reads the first when one dword holds the bytes)
                        const uint32_t* rp = reinterpret_cast<const uint32_t*>(row0 + k * sweep);
                        lo[k] = gfd::ldg(rp);
                        hi[k] = gfd::ldg(rp + (two ? 1 : 0));
                    }
                }
            } else {
#pragma unroll
                for (int k = 0; k < NI; k++) {
                    const int ry = lr + LR * k;
                    lo[k] = hi[k] = 0u;
                    sel[k] = sl;
                    if (lr < LR) {
                        const int yy = gfd::reflect101(min(Y0 + ry - 3, h + 2), h);
                        const uint8_t* row = S + yy * stride + pb;
                        lo[k] = gfd::ldg(reinterpret_cast<const uint32_t*>(row));
                        hi[k] = gfd::ldg(reinterpret_cast<const uint32_t*>(row + (two ? 4 : 0)));
                    }
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < NI; k++) {
                const int ry = lr + LR * k;
                lo[k] = hi[k] = sel[k] = 0u;
                if (lr < LR && ry < BT_R) {
                    const int yy = yin ? Y0 + ry - 3 : gfd::reflect101(min(Y0 + ry - 3, h + 2), h);
                    const uintptr_t row = (uintptr_t)(S + (long long)yy * stride);
                    const uintptr_t base = (row + pmin) & ~(uintptr_t)3;
                    const int o0 = (int)(row + pj[0] - base), o1 = (int)(row + pj[1] - base);
                    const int o2 = (int)(row + pj[2] - base), o3 = (int)(row + pj[3] - base);
                    const bool two = max(max(o0, o1), max(o2, o3)) >= 4;
                    sel[k] = (uint32_t)o0 | (uint32_t)o1 << 8 | (uint32_t)o2 << 16 | (uint32_t)o3 << 24;
                    lo[k] = gfd::ldg(reinterpret_cast<const uint32_t*>(base));
                    hi[k] = gfd::ldg(reinterpret_cast<const uint32_t*>(two ? base + 4 : base));
                }
            }
        }
        uint32_t* s32 = reinterpret_cast<uint32_t*>(&src[0][0]) + lr * (BT_SP / 4) + lq;
#pragma unroll
        for (int k = 0; k < NI; k++)
            if (lr < LR && lr + LR * k < BT_R) s32[LR * (BT_SP / 4) * k] = __builtin_amdgcn_perm(hi[k], lo[k], sel[k]);
    }
    __syncthreads();
    // taps round(256 * gaussian(7, sigma 2)) = 18 34 49 55 49 34 18
    // output x = X0 + 4q + j takes LDS columns 4q + 1 + j .. 4q + 7 + j, i.e.
    // bytes of the row's dwords q, q + 1, q + 2 (w0, w1, w2): per j a chain of
    // v_dot4_u32_u8 with the taps placed at those byte lanes (no realignment)
    constexpr uint32_t T0_0 = 18u << 8 | 34u << 16 | 49u << 24, T0_1 = 55u | 49u << 8 | 34u << 16 | 18u << 24;
    constexpr uint32_t T1_0 = 18u << 16 | 34u << 24, T1_1 = 49u | 55u << 8 | 49u << 16 | 34u << 24, T1_2 = 18u;
    constexpr uint32_t T2_0 = 18u << 24, T2_1 = 34u | 49u << 8 | 55u << 16 | 49u << 24, T2_2 = 34u | 18u << 8;
    constexpr uint32_t T3_1 = 18u | 34u << 8 | 49u << 16 | 55u << 24, T3_2 = 49u | 34u << 8 | 18u << 16;
    // row pass, two source rows per item; a row sum is at most 257 * 255 =
    // 65535, so the two rows share a dword (row 2p low, 2p + 1 high)
    for (int i = tid; i < (BT_R / 2) * (BT_W / 4); i += 256) {
        const int pr = i >> 4, q = i & 15;
        uint4 o;
        auto hsum = [&](int ry, int j) -> uint32_t {
            const uint32_t* r32 = reinterpret_cast<const uint32_t*>(&src[ry][0]) + q;
            const uint32_t w0 = r32[0], w1 = r32[1], w2 = r32[2];
            if (j == 0) return __builtin_amdgcn_udot4(w1, T0_1, __builtin_amdgcn_udot4(w0, T0_0, 0u, false), false);
            if (j == 1)
                return __builtin_amdgcn_udot4(
                    w2, T1_2, __builtin_amdgcn_udot4(w1, T1_1, __builtin_amdgcn_udot4(w0, T1_0, 0u, false), false),
                    false);
            if (j == 2)
                return __builtin_amdgcn_udot4(
                    w2, T2_2, __builtin_amdgcn_udot4(w1, T2_1, __builtin_amdgcn_udot4(w0, T2_0, 0u, false), false),
                    false);
            return __builtin_amdgcn_udot4(w2, T3_2, __builtin_amdgcn_udot4(w1, T3_1, 0u, false), false);
        };
        // low halves of the two rows' sums into one dword (one v_perm_b32)
        o.x = __builtin_amdgcn_perm(hsum(2 * pr + 1, 0), hsum(2 * pr, 0), 0x05040100u);
        o.y = __builtin_amdgcn_perm(hsum(2 * pr + 1, 1), hsum(2 * pr, 1), 0x05040100u);
        o.z = __builtin_amdgcn_perm(hsum(2 * pr + 1, 2), hsum(2 * pr, 2), 0x05040100u);
        o.w = __builtin_amdgcn_perm(hsum(2 * pr + 1, 3), hsum(2 * pr, 3), 0x05040100u);
        *reinterpret_cast<uint4*>(&rows2[pr][4 * q]) = o;
    }
    __syncthreads();
    const int qx = tid & 15, x = X0 + 4 * qx;
    typedef unsigned short gf_u16x2 __attribute__((ext_vector_type(2)));
    auto u2 = [](uint32_t v) { return __builtin_bit_cast(gf_u16x2, v); };
    const gf_u16x2 A0 = {18, 34}, A1 = {49, 55}, A2 = {49, 34}, A3 = {18, 0};  // output row r0
    const gf_u16x2 B0 = {0, 18}, B1 = {34, 49}, B2 = {55, 49}, B3 = {34, 18};  // output row r0 + 1
    auto colv = [&](uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, gf_u16x2 c0, gf_u16x2 c1, gf_u16x2 c2,
                    gf_u16x2 c3) -> uint32_t {
        uint32_t a = __builtin_amdgcn_udot2(u2(p0), c0, 1u << 15, false);
        a = __builtin_amdgcn_udot2(u2(p1), c1, a, false);
        a = __builtin_amdgcn_udot2(u2(p2), c2, a, false);
        a = __builtin_amdgcn_udot2(u2(p3), c3, a, false);
        return min(a >> 16, 255u);
    };
    const uint32_t th2 = (uint32_t)map_th * 0x00010001u;
    uint32_t xm = 0;  // pixels of the quad at least 3 px inside the level, in x
#pragma unroll
    for (int i = 0; i < 4; i++) xm |= (uint32_t)(x + i >= 3 && x + i < w - 3) << i;
    int mask = 0;  // bit 8k + 4r + i: pixel i of the quad in row 32k + r0 + r
#pragma unroll
    for (int k = 0; k < BT_NQ; k++) {
        const int r0 = 2 * (tid >> 4) + 32 * k;
#if BT_SKIP_PAST
        // a wave whose eight rows all lie past the level's last row has no
        // output, no candidate and no score to write (wave-uniform)
        if (Y0 + 32 * k + 8 * (tid >> 6) >= h) continue;
#endif
        // column pass: row pairs r0 / 2 .. + 3 (rows r0 .. r0 + 7) give output
        // rows r0 and r0 + 1, four v_dot2_u32_u16 per pixel (the rounding bias
        // as the accumulator's start)
        uint4 rp[4];
#pragma unroll
        for (int j = 0; j < 4; j++) rp[j] = *reinterpret_cast<const uint4*>(&rows2[(r0 >> 1) + j][4 * qx]);
        uint8_t* D = P.blur + (long long)f * g.bslab + g.boff[l] + (long long)(Y0 + r0) * pw + x;
        const uint32_t a0 = colv(rp[0].x, rp[1].x, rp[2].x, rp[3].x, A0, A1, A2, A3);
        const uint32_t a1 = colv(rp[0].y, rp[1].y, rp[2].y, rp[3].y, A0, A1, A2, A3);
        const uint32_t a2 = colv(rp[0].z, rp[1].z, rp[2].z, rp[3].z, A0, A1, A2, A3);
        const uint32_t a3 = colv(rp[0].w, rp[1].w, rp[2].w, rp[3].w, A0, A1, A2, A3);
        const uint32_t b0 = colv(rp[0].x, rp[1].x, rp[2].x, rp[3].x, B0, B1, B2, B3);
        const uint32_t b1 = colv(rp[0].y, rp[1].y, rp[2].y, rp[3].y, B0, B1, B2, B3);
        const uint32_t b2 = colv(rp[0].z, rp[1].z, rp[2].z, rp[3].z, B0, B1, B2, B3);
        const uint32_t b3 = colv(rp[0].w, rp[1].w, rp[2].w, rp[3].w, B0, B1, B2, B3);
        if (Y0 + r0 < h) *reinterpret_cast<uint32_t*>(D) = a0 | a1 << 8 | a2 << 16 | a3 << 24;
        if (Y0 + r0 + 1 < h) *reinterpret_cast<uint32_t*>(D + pw) = b0 | b1 << 8 | b2 << 16 | b3 << 24;
        // compass pre-test of the quad in rows r0, r0 + 1 (LDS rows r0 + 3, r0 + 4)
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const uint32_t* c32 = reinterpret_cast<const uint32_t*>(&src[r0 + r + 3][0]) + qx;
            const uint32_t L = c32[0], V = c32[1], R = c32[2];
            const uint32_t U = reinterpret_cast<const uint32_t*>(&src[r0 + r][0])[qx + 1];      // dy = -3 (ring 8)
            const uint32_t Dn = reinterpret_cast<const uint32_t*>(&src[r0 + r + 6][0])[qx + 1];  // dy = +3 (ring 0)
            const uint32_t Rt = __builtin_amdgcn_alignbyte(R, V, 3), Lt = __builtin_amdgcn_alignbyte(V, L, 1);
            const uint32_t e = compass2(bytes02(V), bytes02(Dn), bytes02(Rt), bytes02(U), bytes02(Lt), th2);
            const uint32_t o = compass2(bytes13(V), bytes13(Dn), bytes13(Rt), bytes13(U), bytes13(Lt), th2);
            uint32_t m = ((e >> 15) & 1u) | ((o >> 14) & 2u) | ((e >> 29) & 4u) | ((o >> 28) & 8u);
#if defined(GF_BLUR_EXP) && GF_BLUR_EXP == 2
            m &= (uint32_t)(V == 0x12345678u);
#endif
            const int y = Y0 + r0 + r;
            m &= (y >= 3 && y < h - 3) ? xm : 0u;
            mask |= (int)m << (8 * k + 4 * r);
            sco[r0 + r][qx] = 0u;
        }
    }
    int nc;
    int pos = block_scan_256(__popc(mask), scan_tmp, nc);  // its barriers also order the sco zeroing
    while (mask) {
        const int b = __ffs(mask) - 1;
        mask &= mask - 1;
        cand[pos++] = (uint16_t)((2 * (tid >> 4) + 32 * (b >> 3) + ((b >> 2) & 1)) * BT_W + 4 * qx + (b & 3));
    }
    __syncthreads();
    uint8_t* sc8 = reinterpret_cast<uint8_t*>(&sco[0][0]);
#if defined(GF_BLUR_EXP) && GF_BLUR_EXP == 1
    for (int i = tid; i < 0; i += 256) {
#else
    for (int i = tid; i < nc; i += 256) {
#endif
        const int q = cand[i], py = q >> 6, px = q & 63;
        int c[16];
        circle_vals(&src[0][0], BT_SP, px + 4, py + 3, c);
        const int M = fast_max_arc(src[py + 3][px + 4], c);  // corner iff M > th; map entry S + 1 = M
        sc8[q] = M > map_th ? (uint8_t)M : 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < BT_NQ; k++) {
        const int r0 = 2 * (tid >> 4) + 32 * k;
        uint8_t* SC = score + (long long)f * g.bslab + g.boff[l] + (long long)(Y0 + r0) * pw + x;
#pragma unroll
        for (int r = 0; r < 2; r++)
            if (Y0 + r0 + r < h) *reinterpret_cast<uint32_t*>(SC + (long long)r * pw) = sco[r0 + r][qx];
    }
}

// -------------------------------------------------------------- k_fast_cells
// One workgroup per (grid cell, frame). The cell's detection window (the ROI
// minus its 3-px FAST margin, :621) of the score map goes to LDS; corners at
// fast_th survive strict 3x3 non-maximum suppression inside the window
// (neighbours outside it or not corners count 0, as in FAST's row buffers)
// and are listed in row-major order. When at most 3 survive (:623-628) the
// window's map is recomputed at min_th from the unblurred level (the ROI's
// pixels, staged in LDS), suppressed again and the list rewritten.
// NMS: wave w walks rows [w dh/4, (w+1) dh/4) of each 64-column strip, lane =
// column, keeping the three rows it compares in registers (three LDS reads a
// pixel); survivors set their bit in an LDS bit array (bit = row-major pixel
// index). Listing: a workgroup scan over the popcounts of the bit words.
// (Cell windows are at most ~40 px wide, so one strip.)

// sc: the window rows as loaded (row y at byte y * pitch + rsh[y]). Every LDS
// read is unconditional (addresses clamped into the window, out-of-window
// values replaced by 0 afterwards) and each row's base offset is read one
// step before the row itself, so a row step issues its reads together and
// waits once, not once per read.
// BAND: sc holds only window rows [lo, lo + nr) (row nr is the zero row) and
// the rows [yA, yB) of the window are suppressed (k_fast_cells_band).
template <int NWV, bool BAND = false>
__device__ __forceinline__ int cell_nms_bits(const uint8_t* sc, const uint8_t* rsh, int pitch, uint32_t* bits, int dw,
                                             int dh, int th, int yA = 0, int yB = 0, int lo = 0, int nr = 0) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ya = BAND ? yA + wv * (yB - yA) / NWV : wv * dh / NWV;
    const int yb = BAND ? yA + (wv + 1) * (yB - yA) / NWV : (wv + 1) * dh / NWV;
    int cnt = 0;
    // rows outside the window read row dh, a row of zeros with rsh[dh] = 0
    auto rowi = [&](int y) -> int {
        if constexpr (BAND) {
            const int r = y - lo;
            return (y >= 0 && y < dh && r >= 0 && r < nr) ? r : nr;
        } else {
            return (y >= 0 && y < dh) ? y : dh;
        }
    };
    for (int x0 = 0; x0 < dw; x0 += 64) {
        const int x = x0 + lane;
        const bool okc = x < dw;
        // lane masks (all ones inside the window) instead of conditions, so
        // no read is predicated away behind a branch
        const int cl = min(max(x - 1, 0), dw - 1), cc = min(x, dw - 1), cr = min(x + 1, dw - 1);
        // The FAST buffer value at th is S = m - 1 where S >= th, else 0 (m: the
        // map entry S + 1, nonzero only for corners at the map's threshold).
        // Comparisons between such values are comparisons of m on the entries
        // with m > max(th, 1) (m = 1 at th = 0 is a score-0 corner: 0), so each
        // read is one compare against a per-lane bound (255 past the window's
        // edge: every entry reads 0 there, as FAST's row buffers do).
        const int t1 = max(th, 1);
        const int tl = (x >= 1 && x - 1 < dw) ? t1 : 255, tc = okc ? t1 : 255, tr = (x + 1 < dw) ? t1 : 255;
        struct R3 {
            int a, b, c;
        };
        auto row3 = [&](int b) -> R3 {
            const uint8_t* r = sc + b;
            const int va = r[cl], vb = r[cc], vc = r[cr];
            return R3{va > tl ? va : 0, vb > tc ? vb : 0, vc > tr ? vc : 0};
        };
        R3 q[4];
        {
            const int i0 = rowi(ya - 1), i1 = rowi(ya), i2 = rowi(ya + 1);
            q[0] = row3(i0 * pitch + rsh[i0]);
            q[1] = row3(i1 * pitch + rsh[i1]);
            q[2] = row3(i2 * pitch + rsh[i2]);
        }
        int ie = rowi(ya + 2), se = rsh[ie];
        // rows y - 1, y, y + 1 in q[k], q[k + 1], q[k + 2] (mod 4); row y + 2 is
        // read into q[k + 3] one step ahead. Unrolled by four so the roles
        // rotate by register naming, with no moves.
        auto step = [&](int y, R3& u, R3& c, R3& d, R3& e) {
            e = row3(ie * pitch + se);
            const int in = rowi(y + 3);
            se = rsh[in];
            ie = in;
            const int mx = max(max(max(u.a, u.b), max(u.c, c.a)), max(max(c.c, d.a), max(d.b, d.c)));
            const bool keep = okc && c.b != 0 && c.b > mx;
            if (keep) atomicOr(&bits[(y * dw + x) >> 5], 1u << ((y * dw + x) & 31));
            cnt += __popcll(__ballot(keep));
        };
        for (int y = ya; y < yb; y += 4) {
            step(y, q[0], q[1], q[2], q[3]);
            if (y + 1 < yb) step(y + 1, q[1], q[2], q[3], q[0]);
            if (y + 2 < yb) step(y + 2, q[2], q[3], q[0], q[1]);
            if (y + 3 < yb) step(y + 3, q[3], q[0], q[1], q[2]);
        }
    }
    return cnt;  // this wave's survivors
}

// FC_THREADS: workgroup size (64: one wave per cell, no workgroup barrier)
#ifndef FC_THREADS
#define FC_THREADS 256
#endif
constexpr int FC_NT = FC_THREADS, FC_NW = FC_THREADS / 64;
static_assert(FC_NT == 64 || FC_NT == 256 || FC_NT == 512, "k_fast_cells: 1, 4 or 8 waves");

// Exclusive scan of one int per thread across an NW-wave workgroup.
template <int NW>
__device__ int block_scan_nw(int v, int* tmp, int& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int wt;
    const int x = wave_scan_excl(v, wt);
    if (lane == 0) tmp[wid] = wt;
    __syncthreads();
    int base = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        base += i < wid ? tmp[i] : 0;
        total += tmp[i];
    }
    __syncthreads();
    return base + x;
}
__device__ __forceinline__ void fc_sync() {
    if constexpr (FC_NT == 64) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

// k_fast_cells' LDS: the window's score rows realigned to column 0, with a
// zero row above and below and a zero dword either side (the 3x3 NMS reads
// its out-of-window neighbours as 0, as FAST's row buffers hold 0 there);
// survivor bits per window row in whole 32-bit words; the retry's ROI.
struct FcLayout {
    int nq, ndw, pitch, wpr, nwords;
    size_t sc_bytes, bits_bytes, total;
};
__host__ __device__ inline FcLayout fc_layout(int dw, int dh, int w, int h) {
    FcLayout L;
    L.nq = (dw + 3) / 4;  // dwords of window columns per row
    L.ndw = L.nq + 2;
    L.pitch = 4 * L.ndw;
    L.wpr = (dw + 31) / 32;
    L.nwords = dh * L.wpr;
    L.sc_bytes = (size_t)(dh + 2) * L.pitch;
    L.bits_bytes = 4 * (size_t)((L.nwords + 3) & ~3);
    L.total = L.sc_bytes + L.bits_bytes + (size_t)w * h;
    return L;
}

// 3x3 strict NMS over k_fast_cells' realigned window, four columns per lane
// (lane L: columns 4L .. 4L + 3) on packed 16-bit lanes: per row the dwords
// L - 1, L, L + 1 give the even columns E = (4L, 4L + 2), the odd O = (4L + 1,
// 4L + 3) and their left / right neighbour pairs EL = (4L - 1, 4L + 1), OR =
// (4L + 2, 4L + 4). The map entries m count only when m > t1 = max(th, 1)
// (FAST's buffer value at th, see cell_nms_bits): m' = sat(m - t1) keeps their
// order and sends the others to 0, so "m > every counted neighbour and m
// counted" is m' > the neighbours' max m'. Wave w takes window rows [w dh / NW,
// (w + 1) dh / NW); one pass covers 256 columns. Returns the wave's survivors.
template <int NWV>
__device__ __forceinline__ int cell_nms4(const uint32_t* sc32, const FcLayout& Ly, uint32_t* bits, int dh, int th) {
    typedef unsigned short u2 __attribute__((ext_vector_type(2)));
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ya = wv * dh / NWV, yb = (wv + 1) * dh / NWV;
    const unsigned short t1 = (unsigned short)max(th, 1);
    const u2 T = {t1, t1}, ONE = {1, 1};
    auto U = [](uint32_t v) { return __builtin_bit_cast(u2, v); };
    struct Q {
        u2 e, o, el, orr;
    };
    int cnt = 0;
    for (int L0 = 0; L0 < Ly.nq; L0 += 64) {
        const int L = L0 + lane;
        const bool okq = L < Ly.nq;
        const uint32_t* col = sc32 + min(L, Ly.nq - 1);  // clamped lanes read the row's last words (dropped)
        auto rowq = [&](int r) -> Q {  // LDS row r = window row r - 1
            const uint32_t* q = col + r * Ly.ndw;
            const uint32_t a = q[0], b = q[1], c = q[2];
            Q x;
            x.e = __builtin_elementwise_sub_sat(U(__builtin_amdgcn_perm(0u, b, 0x0c020c00u)), T);
            x.o = __builtin_elementwise_sub_sat(U(__builtin_amdgcn_perm(0u, b, 0x0c030c01u)), T);
            x.el = __builtin_elementwise_sub_sat(U(__builtin_amdgcn_perm(a, b, 0x0c010c07u)), T);
            x.orr = __builtin_elementwise_sub_sat(U(__builtin_amdgcn_perm(c, b, 0x0c040c02u)), T);
            return x;
        };
        uint32_t* brow = bits + ya * Ly.wpr + (L >> 3);
        const int sh = 4 * (L & 7);
        // rows y - 1, y, y + 1 in u, c, d; unrolled by three so the roles
        // rotate by naming
        auto step = [&](int y, const Q& u, const Q& c, Q& d) {
            d = rowq(y + 2);
            const u2 vE = __builtin_elementwise_max(u.e, d.e), vO = __builtin_elementwise_max(u.o, d.o);
            const u2 vEL = __builtin_elementwise_max(u.el, d.el), vOR = __builtin_elementwise_max(u.orr, d.orr);
            const u2 mxE = __builtin_elementwise_max(__builtin_elementwise_max(vE, vEL),
                                                     __builtin_elementwise_max(vO, __builtin_elementwise_max(c.el, c.o)));
            const u2 mxO = __builtin_elementwise_max(__builtin_elementwise_max(vO, vOR),
                                                     __builtin_elementwise_max(vE, __builtin_elementwise_max(c.e, c.orr)));
            const u2 kE = __builtin_elementwise_min(__builtin_elementwise_sub_sat(c.e, mxE), ONE);
            const u2 kO = __builtin_elementwise_min(__builtin_elementwise_sub_sat(c.o, mxO), ONE);
            const uint32_t t = __builtin_bit_cast(uint32_t, kE) | (__builtin_bit_cast(uint32_t, kO) << 1);
            const uint32_t m = okq ? ((t & 3u) | ((t >> 14) & 12u)) : 0u;  // bit i: column 4L + i
            if (m) atomicOr(brow + (y - ya) * Ly.wpr, m << sh);
            cnt += __popc(m);
        };
        Q q0 = rowq(ya), q1 = rowq(ya + 1), q2;
        for (int y = ya; y < yb; y += 3) {
            step(y, q0, q1, q2);
            if (y + 1 < yb) step(y + 1, q1, q2, q0);
            if (y + 2 < yb) step(y + 2, q2, q0, q1);
        }
    }
    return gfd::warp_sum(cnt);
}

template <typename E>
__global__ __launch_bounds__(FC_NT) void k_fast_cells(Planes P, LevelGeom g, const uint8_t* __restrict__ score,
                                                    const CellInfo* __restrict__ cells, E* __restrict__ lists,
                                                    long long list_stride, int* __restrict__ counts, int fast_th,
                                                    int min_th) {
    gfd::ext_prio();
    extern __shared__ __align__(16) uint8_t smem[];
    __shared__ int s_cnt[2][FC_NW];
    __shared__ int scan_tmp[FC_NW];
    int cid, f;
    gfd::xcd_block(cid, f);
    const int tid = threadIdx.x;
    const CellInfo ci = cells[cid];
    if (ci.band) return;  // a window past this kernel's LDS: k_fast_cells_band
    const int dw = ci.w - 6, dh = ci.h - 6;
    if (!ci.valid || dw <= 0 || dh <= 0) {  // degenerate ROI: FAST finds nothing
        if (tid == 0) counts[(long long)f * g.ncells + cid] = 0;
        return;
    }
    const FcLayout Ly = fc_layout(dw, dh, ci.w, ci.h);
    uint8_t* sc = smem;  // window row y, column x at (y + 1) * pitch + 4 + x
    uint32_t* sc32 = reinterpret_cast<uint32_t*>(smem);
    uint32_t* bits = reinterpret_cast<uint32_t*>(smem + Ly.sc_bytes);  // window row y: words y * wpr ..
    const int l = ci.level, lw = g.pw[l];
    const uint8_t* SC = score + (long long)f * g.bslab + g.boff[l] + (long long)(ci.y0 + 3) * lw + ci.x0 + 3;
    {  // the window realigned: every row of the pitched map has SC's byte shift.
        // Thread t owns LDS dword column j = t % ndw of rows t / ndw + k rstep,
        // so a row's address is one step from the last (no index split per load)
        const uint32_t sh = (uint32_t)((uintptr_t)SC & 3u);
        const uint32_t* SCa = reinterpret_cast<const uint32_t*>((uintptr_t)SC & ~(uintptr_t)3);
        const int lw4 = lw >> 2, nrows = dh + 2;
        const int ndw = Ly.ndw, rstep = max(FC_NT / ndw, 1);
        const int j = tid % ndw, r0 = tid / ndw;
        const bool jdata = j >= 1 && j <= Ly.nq;
        uint32_t bmask = ~0u;  // the window's bytes of this dword column
        if (jdata && dw - 4 * (j - 1) < 4) bmask = (1u << (8 * (dw - 4 * (j - 1)))) - 1u;
        constexpr int FC_LB = 8;  // rows per thread in flight
        for (int rb = r0; rb < nrows; rb += FC_LB * rstep) {  // ndw <= FC_NT (host: wider windows go to k_fast_cells_band)
            // loads unconditional at clamped (in-window) addresses, the pads
            // selected after them: a load behind a branch would have its
            // result merged before the next one issues (a wait per row)
            uint32_t lo[FC_LB], hi[FC_LB];
            const int jc = min(max(j, 1), Ly.nq) - 1;
#pragma unroll
            for (int k = 0; k < FC_LB; k++) {
                const int rc = min(max(rb + k * rstep, 1), dh) - 1;
                const uint32_t* src = SCa + (long long)rc * lw4 + jc;
                lo[k] = gfd::ldg(src);
                hi[k] = gfd::ldg(src + 1);
            }
#pragma unroll
            for (int k = 0; k < FC_LB; k++) {
                const int r = rb + k * rstep;
                const bool data = jdata && r >= 1 && r <= dh;
                if (r < nrows && r0 < rstep)
                    sc32[r * ndw + j] = data ? __builtin_amdgcn_alignbyte(hi[k], lo[k], sh) & bmask : 0u;
            }
        }
    }
    for (int i = tid; i < Ly.nwords; i += FC_NT) bits[i] = 0;
    fc_sync();
    int c = cell_nms4<FC_NW>(sc32, Ly, bits, dh, fast_th);
    if ((tid & 63) == 0) s_cnt[0][tid >> 6] = c;
    fc_sync();
    int total = 0;
#pragma unroll
    for (int k = 0; k < FC_NW; k++) total += s_cnt[0][k];
    if (total <= 3) {  // ORBextractor.cc:623-628: retry with the minimum threshold
        // the ROI (window + 3-px ring margin) of the unblurred level to LDS
        uint8_t* roi = smem + Ly.sc_bytes + Ly.bits_bytes;
        int sstride;
        const uint8_t* Sl = level_plane(P, g, f, l, sstride) + (long long)ci.y0 * sstride + ci.x0;
        for (int i = tid; i < ci.w * ci.h; i += FC_NT) {
            const int r = pyr_div(i, 1.0f / (float)ci.w);
            roi[i] = gfd::ldg(Sl + (long long)r * sstride + (i - r * ci.w));
        }
        fc_sync();
        for (int i = tid; i < dw * dh; i += FC_NT) {
            const int y = pyr_div(i, 1.0f / (float)dw), x = i - y * dw;
            int cv[16];
            circle_vals(roi, ci.w, x + 3, y + 3, cv);
            const int M = fast_max_arc(roi[(y + 3) * ci.w + x + 3], cv);
            sc[(y + 1) * Ly.pitch + 4 + x] = M > min_th ? (uint8_t)M : 0;
        }
        for (int i = tid; i < Ly.nwords; i += FC_NT) bits[i] = 0;
        fc_sync();
        c = cell_nms4<FC_NW>(sc32, Ly, bits, dh, min_th);
        if ((tid & 63) == 0) s_cnt[1][tid >> 6] = c;
        fc_sync();
        total = 0;
#pragma unroll
        for (int k = 0; k < FC_NW; k++) total += s_cnt[1][k];
    }
    E* out = lists + (long long)f * list_stride + ci.cap_off;
    const int X0 = ci.x0 + 3, Y0 = ci.y0 + 3;
    int base = 0;
    for (int w0 = 0; w0 < Ly.nwords; w0 += FC_NT) {  // words in row-major order: the survivors in FAST's order
        const int i = w0 + tid;
        uint32_t word = i < Ly.nwords ? bits[i] : 0u;
        int tot;
        int off;
        if constexpr (FC_NT == 64) {
            off = base + wave_scan_excl(__popc(word), tot);
        } else {
            off = base + block_scan_nw<FC_NW>(__popc(word), scan_tmp, tot);
        }
        if (word) {
            const int y = i / Ly.wpr, xw = 32 * (i - y * Ly.wpr);
            const uint8_t* srow = sc + (y + 1) * Ly.pitch + 4;
            while (word) {
                const int x = xw + __ffs(word) - 1;
                word &= word - 1;
                out[off++] = cell_entry<E>(srow[x] - 1, X0 + x, Y0 + y, P, g, f, l);
            }
        }
        base += tot;
    }
    if (tid == 0) counts[(long long)f * g.ncells + cid] = total;
}

// One 256-thread workgroup per (large cell, frame): a cell window whose score
// rows (and, for the minimum-threshold retry, ROI rows) do not fit
// k_fast_cells' LDS — small nFeatures make few, large cells (ORBextractor.cc
// :540-560 grids any level). The same FAST / NMS / listing as k_fast_cells,
// with the window walked in bands of ci.band rows: each band's rows plus one
// halo row either side go to LDS (the halo rows are what the 3x3 NMS of the
// band's edge rows reads), the survivor bits of the whole window stay in LDS,
// and the listing reads each survivor's score again from the map (or
// recomputes it from the level on the retry pass).
template <typename E>
__global__ __launch_bounds__(256) void k_fast_cells_band(Planes P, LevelGeom g, const uint8_t* __restrict__ score,
                                                         const CellInfo* __restrict__ cells,
                                                         const int* __restrict__ band_ids, E* __restrict__ lists,
                                                         long long list_stride, int* __restrict__ counts, int fast_th,
                                                         int min_th) {
    gfd::ext_prio();
    extern __shared__ __align__(16) uint8_t smem[];
    __shared__ int s_cnt[4];
    __shared__ int scan_tmp[4];
    const int cid = band_ids[blockIdx.x], f = blockIdx.y, tid = threadIdx.x;
    const CellInfo ci = cells[cid];
    const int dw = ci.w - 6, dh = ci.h - 6, BH = ci.band;
    const int n = dw * dh, nwords = (n + 31) >> 5;
    const int ndw = (dw + 6) >> 2, pitch = 4 * ndw;
    uint32_t* bits = reinterpret_cast<uint32_t*>(smem);
    uint8_t* sc = smem + 16 * ((nwords + 3) / 4);              // (BH + 3) rows x pitch
    uint8_t* rsh = sc + (BH + 3) * pitch;                      // BH + 3 row shifts
    uint8_t* roi = rsh + ((BH + 3 + 15) & ~15);                // (BH + 8) ROI rows x ci.w (retry)
    const int l = ci.level, lw = g.pw[l];
    const uint8_t* SC = score + (long long)f * g.bslab + g.boff[l] + (long long)(ci.y0 + 3) * lw + ci.x0 + 3;
    int sstride;
    const uint8_t* Sl = level_plane(P, g, f, l, sstride) + (long long)ci.y0 * sstride + ci.x0;
    int total = 0, pass = 0;
    for (; pass < 2; pass++) {
        const int th = pass ? min_th : fast_th;
        for (int i = tid; i < nwords; i += 256) bits[i] = 0;
        total = 0;
        for (int yb = 0; yb < dh; yb += BH) {
            const int ye = min(yb + BH, dh), lo = max(yb - 1, 0), hi = min(ye + 1, dh), nr = hi - lo;
            __syncthreads();  // the previous band's NMS reads are done
            if (pass == 0) {
                for (int i = tid; i < nr * ndw; i += 256) {
                    const int r = pyr_div(i, 1.0f / (float)ndw), q = i - r * ndw;
                    const uintptr_t a = (uintptr_t)(SC + (long long)(lo + r) * lw);
                    uint32_t v = 0;
                    if (4 * q < (int)(a & 3) + dw) v = gfd::ldg(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3) + q);
                    reinterpret_cast<uint32_t*>(sc)[i] = v;
                }
                for (int r = tid; r < nr; r += 256) rsh[r] = (uint8_t)((uintptr_t)(SC + (long long)(lo + r) * lw) & 3);
            } else {
                // window row y's circle lies in ROI rows y .. y + 6
                const int rr = nr + 6;
                for (int i = tid; i < rr * ci.w; i += 256) {
                    const int r = pyr_div(i, 1.0f / (float)ci.w);
                    roi[i] = gfd::ldg(Sl + (long long)(lo + r) * sstride + (i - r * ci.w));
                }
                __syncthreads();
                for (int i = tid; i < nr * dw; i += 256) {
                    const int y = pyr_div(i, 1.0f / (float)dw), x = i - y * dw;
                    int c[16];
                    circle_vals(roi, ci.w, x + 3, y + 3, c);
                    const int M = fast_max_arc(roi[(y + 3) * ci.w + x + 3], c);
                    sc[y * pitch + x] = M > min_th ? (uint8_t)M : 0;
                }
                for (int r = tid; r < nr; r += 256) rsh[r] = 0;
            }
            if (tid == 0) rsh[nr] = 0;
            for (int i = tid; i < ndw; i += 256) reinterpret_cast<uint32_t*>(sc + nr * pitch)[i] = 0u;
            __syncthreads();
            const int c = cell_nms_bits<4, true>(sc, rsh, pitch, bits, dw, dh, th, yb, ye, lo, nr);
            if ((tid & 63) == 0) s_cnt[tid >> 6] = c;
            __syncthreads();
            total += s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        }
        if (total > 3) break;  // else ORBextractor.cc:623-628: retry with the minimum threshold
    }
    if (pass == 2) pass = 1;
    __syncthreads();
    E* out = lists + (long long)f * list_stride + ci.cap_off;
    const int X0 = ci.x0 + 3, Y0 = ci.y0 + 3;
    int base = 0;
    for (int w0 = 0; w0 < nwords; w0 += 256) {
        const int i = w0 + tid;
        uint32_t word = i < nwords ? bits[i] : 0u;
        int tot;
        int off = base + block_scan_nw<4>(__popc(word), scan_tmp, tot);
        while (word) {
            const int p = 32 * i + __ffs(word) - 1;
            word &= word - 1;
            const int y = pyr_div(p, 1.0f / (float)dw), x = p - y * dw;
            int S;
            if (pass == 0) {
                S = SC[(long long)y * lw + x] - 1;
            } else {
                int c[16];
                circle_vals(Sl, sstride, x + 3, y + 3, c);
                S = fast_max_arc(Sl[(long long)(y + 3) * sstride + x + 3], c) - 1;
            }
            out[off++] = cell_entry<E>(S, X0 + x, Y0 + y, P, g, f, l);
        }
        base += tot;
    }
    if (tid == 0) counts[(long long)f * g.ncells + cid] = total;
}

// -------------------------------------------------------------- k_select
// One workgroup per (level, frame). KeyPointsFilter::retainBest is
// std::nth_element (libstdc++ __introselect: median-of-three pivot, unguarded
// Hoare partition, heap_select past the depth limit, insertion sort below 4),
// and the keypoint order it leaves is what every later stage sees, so each
// selection replays it exactly — one wave per list, the list in LDS:
//   * the pivot choice, the depth bookkeeping and the small-range insertion
//     sort run on lane 0 (O(1) per round);
//   * the partition runs on all 64 lanes. __unguarded_partition swaps the k-th
//     element from the left that is not better than the pivot with the k-th
//     element from the right that is not worse, for every k while the left
//     one lies before the right one (the swapped elements act as sentinels, so
//     the scans never see a swapped position before that condition fails);
//     it returns min(L_k*, R_{k*-1}) for the first failing k*. The two
//     stopper position lists come from ballots over 64-element windows, k*
//     from one more ballot pass (L_k < R_k is monotone in k), the swaps are
//     disjoint.
// Lists longer than the LDS buffer fall back to the sequential replay on
// global memory (gfsel::retain_best_truncate, same result).
#define SEL_MAX_CELLS 1024
#ifndef SEL_THREADS
#define SEL_THREADS 512
#endif
#define SEL_BUF 1024  // entries of wave 0's buffer (cell lists and the level list)
// entries of the other waves' buffers (cell lists only). 512 since r04: the
// workgroup's LDS drops from 77 to 49 KB, so it fits beside the tracking
// kernels' workgroups (k_select 0.46 -> 0.38 ms per launch in the step,
// 101.1-101.8k -> 101.4-102.4k frames/s, profiles/r04/ab8_*.json, ab9_*.json);
// the rare cell list above 512 entries that needs a cut waits for wave 0's
// 1024-entry buffer (exact either way; the c256 build's tests cover it)
#ifndef SEL_BUF_CELL
#define SEL_BUF_CELL 512
#endif
// one wave's LDS list and partition scratch; wave 0's is SEL_BUF long, the
// others' SEL_BUF_CELL (a cell's corners after NMS rarely pass 100), so the
// workgroup takes 8 + 7 x 2 KB instead of 8 x 8 KB and more fit a CU
template <typename E>
struct SelWave {
    E* a;
    uint16_t *lp, *rp;
    int cap;
};
template <typename E>
constexpr size_t sel_wave_bytes(int cap) { return (size_t)cap * (sizeof(E) + 2 * sizeof(uint16_t)); }
template <typename E>
constexpr size_t sel_wave_lds() {
    return sel_wave_bytes<E>(SEL_BUF) + (SEL_THREADS / 64 - 1) * sel_wave_bytes<E>(SEL_BUF_CELL);
}
// + the per-cell counts, quotas, offsets and flags of a level (maxnc cells at most)
template <typename E>
constexpr size_t sel_lds(int maxnc) { return sel_wave_lds<E>() + sizeof(int) * (3 * (size_t)maxnc + 1) + (size_t)maxnc; }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename E>
__device__ __forceinline__ int sel_resp(E e) { return Ent<E>::key(e); }

// __unguarded_partition(a + lo, a + hi, a + pivot) with KeypointResponseGreater.
template <typename E>
__device__ __forceinline__ int wave_partition(const SelWave<E>& W, int lo, int hi, int P) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int nL = 0, nR = 0;
    for (int i0 = 0; i0 < hi - lo; i0 += 64) {
        const int i = lo + i0 + lane, j = hi - 1 - i0 - lane;
        const bool sl = i < hi && !(sel_resp(W.a[i]) > P);  // left scan stops: not better than the pivot
        const bool sr = j >= lo && !(P > sel_resp(W.a[j]));  // right scan stops: not worse
        const unsigned long long bl = __ballot(sl), br = __ballot(sr);
        if (sl) W.lp[nL + __popcll(bl & lt)] = (uint16_t)i;
        if (sr) W.rp[nR + __popcll(br & lt)] = (uint16_t)j;
        nL += __popcll(bl);
        nR += __popcll(br);
    }
    wave_sync();
    const int m = min(nL, nR);
    int ks = 0;
    for (int k0 = 0; k0 < m; k0 += 64) {
        const int k = k0 + lane;
        const unsigned long long ok = __ballot(k < m && W.lp[k] < W.rp[k]);
        ks += __popcll(ok);
        if (~ok & ((k0 + 64 <= m) ? ~0ull : ((1ull << (m - k0)) - 1ull))) break;  // monotone: done
    }
    for (int k = lane; k < ks; k += 64) {
        const int x = W.lp[k], y = W.rp[k];
        const E ax = W.a[x], ay = W.a[y];
        W.a[x] = ay;
        W.a[y] = ax;
    }
    const int Lk = ks < nL ? (int)W.lp[ks] : hi;
    const int Rk = ks > 0 ? (int)W.rp[ks - 1] : hi;
    wave_sync();
    return min(Lk, Rk);
}

// std::nth_element(a, a + nth, a + n) on the wave's LDS list, all lanes.
template <typename E>
__device__ __forceinline__ void wave_nth_element(const SelWave<E>& W, int nth, int n) {
    const int lane = threadIdx.x & 63;
    const EntGreater<E> comp;
    if (n == 0 || nth == n) return;
    int first = 0, last = n;
    int depth = 2 * gfsel::lg_(n);
    while (last - first > 3) {
        if (depth == 0) {
            if (lane == 0) {
                gfsel::heap_select(W.a, first, nth + 1, last, comp);
                gfsel::swap_(W.a[first], W.a[nth]);
            }
            wave_sync();
            return;
        }
        --depth;
        const int mid = first + (last - first) / 2;
        if (lane == 0) gfsel::move_median_to_first(W.a, first, first + 1, mid, last - 1, comp);
        wave_sync();
        const int cut = wave_partition(W, first + 1, last, sel_resp(W.a[first]));
        if (cut <= nth)
            first = cut;
        else
            last = cut;
    }
    if (lane == 0) gfsel::insertion_sort(W.a, first, last, comp);
    wave_sync();
}

// dst[0 .. n) = src[0 .. n) by one wave, 8 loads per lane in flight before
// their stores (a plain strided loop waits for every load before the next)
template <typename E, typename D>
__device__ __forceinline__ void wave_copy_in(D* dst, const E* src, int n) {
    const int lane = threadIdx.x & 63;
    constexpr int CB = 8;
    for (int i0 = 0; i0 < n; i0 += 64 * CB) {
        E v[CB];
#pragma unroll
        for (int k = 0; k < CB; k++) {
            const int i = i0 + 64 * k + lane;
            v[k] = i < n ? src[i] : (E)0;
        }
#pragma unroll
        for (int k = 0; k < CB; k++) {
            const int i = i0 + 64 * k + lane;
            if (i < n) dst[i] = v[k];
        }
    }
}

// retainBest(list, keep) + truncation, written to dst[0 .. keep): one wave.
template <typename E>
__device__ __forceinline__ void wave_retain_to(const SelWave<E>& W, E* list, int n, int keep, E* dst) {
    const int lane = threadIdx.x & 63;
    if (keep <= 0) return;
    if (n <= keep) {
        wave_copy_in(dst, list, n);
        return;
    }
    if (n > W.cap) {  // sequential replay on global memory
        if (lane == 0) gfsel::retain_best_truncate(list, n, keep, EntGreater<E>());
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (int i = lane; i < keep; i += 64) dst[i] = list[i];
        return;
    }
    wave_copy_in(W.a, list, n);
    wave_sync();
    wave_nth_element(W, keep - 1, n);
    for (int i = lane; i < keep; i += 64) dst[i] = W.a[i];
}

// Quota redistribution of one level (ORBextractor.cc:673-721) by one wave:
// each round is a per-cell map with integer sums (order-free), so the rounds
// give the sequential loop's nToRetain exactly. Cells skipped by the ROI loop
// (valid == 0) keep nTotal = 0, nToRetain = 0, bNoMore = false. Leaves keep[c]
// and off[c] = exclusive prefix of the kept counts (off[nc] = the level's
// total) in the wave's LDS arrays; cnt[c] = the cell's corner count.
__device__ void wave_quota(const int* __restrict__ counts, const CellInfo* __restrict__ cells, int nc, int nf,
                           int* cnt, int* keep, int* off, uint8_t* flag) {
    const int lane = threadIdx.x & 63;
    int dist = 0, nomore = 0;
    for (int c = lane; c < nc; c += 64) {
        const int n = counts[c];
        const bool v = cells[c].valid != 0;
        cnt[c] = v ? n : 0;
        int k = 0, fl = 0;
        if (!v) {
            k = -1;  // not a cell of the ROI loop: no quota, no list
        } else if (n > nf) {
            k = nf;
        } else {
            k = n;
            dist += nf - n;
            fl = 1;
            nomore++;
        }
        keep[c] = k;
        flag[c] = (uint8_t)fl;
    }
    int nToDistribute = gfd::warp_sum(dist), nNoMore = gfd::warp_sum(nomore);
    while (nToDistribute > 0 && nNoMore < nc) {
        const int nNew = nf + (int)ceilf((float)nToDistribute / (float)(nc - nNoMore));
        dist = 0;
        nomore = 0;
        for (int c = lane; c < nc; c += 64) {
            if (flag[c]) continue;  // (skipped cells take part: nTotal 0, bNoMore false)
            const int n = cnt[c];
            if (n > nNew) {
                if (keep[c] >= 0) keep[c] = nNew;
            } else {
                if (keep[c] >= 0) keep[c] = n;
                dist += nNew - n;
                flag[c] = 1;
                nomore++;
            }
        }
        nToDistribute = gfd::warp_sum(dist);
        nNoMore += gfd::warp_sum(nomore);
    }
    // keep[c] <= cnt[c], so retainBest leaves exactly keep[c] per cell (:734-736)
    int base = 0;
    for (int c0 = 0; c0 < nc; c0 += 64) {
        const int c = c0 + lane;
        const int v = c < nc && keep[c] > 0 ? keep[c] : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (c < nc) off[c] = base + x - v;
        base += __shfl(x, 63, 64);
    }
    if (lane == 0) off[nc] = base;
    wave_sync();
}

// retainBest per cell: one wave per (cell, frame), every cell of every level
// at once (cells of a level no longer queue behind one workgroup's waves).
// The wave redoes its level's quota (a few integer rounds over the level's
// cells) and writes its cell's kept entries at the cell's offset in the level
// list. The level's first cell also records the level total for k_select_level.
#define SEL_CW 4  // cell waves per workgroup
template <typename E>
constexpr size_t sel_cell_wave_lds(int maxnc) {
    return sel_wave_bytes<E>(SEL_BUF) + sizeof(int) * (3 * (size_t)maxnc + 1) + (((size_t)maxnc + 15) & ~(size_t)15);
}

template <typename E>
__global__ __launch_bounds__(64 * SEL_CW) void k_select_cells(LevelGeom g, const CellInfo* __restrict__ cells,
                                                              E* __restrict__ lists, long long list_stride,
                                                              const int* __restrict__ counts,
                                                              E* __restrict__ lvl_lists, long long lvl_stride,
                                                              int* __restrict__ lvl_counts, int maxnc) {
    gfd::ext_prio();
    extern __shared__ __align__(16) uint8_t sel_dyn[];
    const int f = blockIdx.y, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = blockIdx.x * SEL_CW + wv;  // cell (all levels, level-major)
    if (c >= g.ncells) return;               // whole wave
    uint8_t* base = sel_dyn + (size_t)wv * sel_cell_wave_lds<E>(maxnc);
    SelWave<E> W;
    W.a = reinterpret_cast<E*>(base);
    W.lp = reinterpret_cast<uint16_t*>(W.a + SEL_BUF);
    W.rp = W.lp + SEL_BUF;
    W.cap = SEL_BUF;
    int* cnt = reinterpret_cast<int*>(base + sel_wave_bytes<E>(SEL_BUF));
    int* keep = cnt + maxnc;
    int* off = keep + maxnc;  // maxnc + 1
    uint8_t* flag = reinterpret_cast<uint8_t*>(off + maxnc + 1);
    const CellInfo me = cells[c];  // level and list offset in one load batch (the list address waits on nothing else)
    const int l = me.level;
    const int cb = g.cell_begin[l], nc = g.cell_begin[l + 1] - cb, ci = c - cb;
    wave_quota(counts + (long long)f * g.ncells + cb, cells + cb, nc, g.nfcell[l], cnt, keep, off, flag);
    E* L = lvl_lists + (long long)f * lvl_stride + g.lvl_off[l];
    if (ci == 0 && lane == 0) lvl_counts[(long long)f * g.nlevels + l] = off[nc];
    if (keep[ci] > 0) {
        E* a = lists + (long long)f * list_stride + me.cap_off;
        wave_retain_to(W, a, cnt[ci], keep[ci], L + off[ci]);
    }
}

// The level's retainBest (:750-752) on the concatenated cell lists: one wave
// per (frame, level); total from k_select_cells, the cut count back in place.
template <typename E>
__global__ __launch_bounds__(64) void k_select_level(LevelGeom g, E* __restrict__ lvl_lists, long long lvl_stride,
                                                     int* __restrict__ lvl_counts) {
    gfd::ext_prio();
    extern __shared__ __align__(16) uint8_t sel_dyn[];
    const int f = blockIdx.x, l = blockIdx.y, lane = threadIdx.x;
    SelWave<E> W;
    W.a = reinterpret_cast<E*>(sel_dyn);
    W.lp = reinterpret_cast<uint16_t*>(W.a + SEL_BUF);
    W.rp = W.lp + SEL_BUF;
    W.cap = SEL_BUF;
    E* L = lvl_lists + (long long)f * lvl_stride + g.lvl_off[l];
    int* out = lvl_counts + (long long)f * g.nlevels + l;
    const int total = *out, nd = g.ndesired[l];
    if (nd >= 0 && total > nd && nd > 0 && total <= SEL_BUF) {
        wave_copy_in(W.a, L, total);
        wave_sync();
        wave_nth_element(W, nd - 1, total);
        for (int i = lane; i < nd; i += 64) L[i] = W.a[i];
    } else if (lane == 0) {
        gfsel::retain_best_truncate(L, total, nd, EntGreater<E>());
    }
    if (lane == 0) *out = (nd < 0 || total <= nd) ? total : nd;
}

// -------------------------------------------------------------- k_describe
__device__ float fast_atan2f(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// One wave per keypoint, 4 per workgroup.
// Per wave: the 31x31 IC_Angle patch of the unblurred level and the 37x37
// window of the blurred level that holds every rotated rBRIEF sample (the
// pattern's points lie within 18.4 px of the keypoint), both fetched as
// aligned dwords in one batch right after the keypoint entry, so a keypoint
// costs two dependent memory round trips. A keypoint whose window leaves the
// level reads its rBRIEF samples from HBM with the reflect-101 border instead.
#define DS_IC 31
#define DS_ICW 9    // dwords per IC row (31 bytes at any alignment)
#define DS_BL 37
#define DS_BLW 10   // dwords per window row (37 bytes at any alignment)
#define DS_LOADS ((DS_IC * DS_ICW + DS_BL * DS_BLW + 63) / 64)
// rBRIEF samples read as aligned 8-byte words (ds_read_b64 banks over 64
// dwords, not 32: the half-wave's pseudo-random sample positions collide on a
// bank half as often) with the byte picked by a shift
#ifndef DESC_B64
#define DESC_B64 0
#endif
struct __align__(8) DescLds {
    uint32_t bl[DS_BL * DS_BLW];  // first: 8-byte aligned (1480 B)
    uint32_t ic[DS_IC * DS_ICW];
    uint8_t ic_sh[DS_IC];
};

// Two keypoints per wave, one per 32-lane half: the halves' loads go out in
// the same batch, so a wave covers two keypoints with the same two round trips.
__device__ __forceinline__ int half_sum(int v) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);  // xor < 32 stays inside the half
    return v;
}

template <typename E>
__global__ __launch_bounds__(256) void k_describe(Planes P, LevelGeom g, const E* __restrict__ lvl_lists,
                                                  long long lvl_stride, const int* __restrict__ lvl_counts,
                                                  gf_keypoint* __restrict__ kps, uint8_t* __restrict__ desc,
                                                  int* __restrict__ out_counts, int cap) {
    gfd::ext_prio();
    __shared__ DescLds sh_all[8];
    // the rBRIEF pattern, one dword per test, bit-major (test 8 i + bit at
    // bit * 32 + i): the 32 lanes of a half read 32 consecutive dwords
    __shared__ uint32_t sh_pat[256];
    __shared__ uint32_t sh_ictab[256];  // IC_Angle's row weights and masks (c_ic_tab)
    int bx, f;
    gfd::xcd_block(bx, f);
    int cnt[GF_MAX_LEVELS];  // all level counts in one batch of loads, in flight with the tables'
#pragma unroll
    for (int i = 0; i < GF_MAX_LEVELS; i++) cnt[i] = lvl_counts[(long long)f * g.nlevels + min(i, g.nlevels - 1)];
    sh_pat[(threadIdx.x & 7) * 32 + (threadIdx.x >> 3)] = c_pattern8[threadIdx.x];
    sh_ictab[threadIdx.x] = c_ic_tab[threadIdx.x];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < GF_MAX_LEVELS; i++) cnt[i] = i < g.nlevels ? cnt[i] : 0;
    const int lane = threadIdx.x & 63, hl = lane & 31, half = (threadIdx.x >> 5);  // half = slot 0..7
    DescLds& W = sh_all[half];
    const int k = bx * 8 + half;
    int total = 0, l = -1, idx = 0;
#pragma unroll
    for (int i = 0; i < GF_MAX_LEVELS; i++) {
        if (l < 0 && i < g.nlevels && k < total + cnt[i]) {
            l = i;
            idx = k - total;
        }
        total += cnt[i];
    }
    if (k == 0 && hl == 0) out_counts[f] = total;
    if (__ballot(l >= 0) == 0) return;  // whole wave past the last keypoint
    const bool live = l >= 0;
    const int lv = live ? l : 0;
    const E e = live ? lvl_lists[(long long)f * lvl_stride + g.lvl_off[lv] + idx] : (E)0;
    const int x = (int)(e & 0xfff), y = (int)((e >> 12) & 0xfff);
    const int w = g.w[lv], h = g.h[lv], pwl = g.pw[lv];
    int stride;
    const uint8_t* Pl = level_plane(P, g, f, lv, stride);
    const uint8_t* B = P.blur + (long long)f * g.bslab + g.boff[lv];
    const bool win = live && x >= 18 && x + 18 < w && y >= 18 && y + 18 < h;

    {  // one batch: IC rows y-15..y+15 (cols x-15..), window rows y-18..y+18 (cols x-18..)
        // Each lane owns one dword column of every third row, so a load's
        // address is one multiply-add from the lane's column base (the flat
        // index split by division cost ~13 VALU per load, a third of the
        // kernel's VALU). IC: lanes (rg, q) = (hl / 9, hl % 9) for hl < 27, rows
        // rg + 3 k; window: (hl / 10, hl % 10) for hl < 30, rows rg + 3 k.
        // Lanes past them, and rows past the last, repeat the last lane's
        // column / the last row: they load and store the same words again.
        constexpr int NI = (DS_IC + 2) / 3, NB = (DS_BL + 2) / 3;
        const int hq = min(hl, 3 * DS_ICW - 1), rg = hq / DS_ICW, q = hq - rg * DS_ICW;
        const int hw = min(hl, 3 * DS_BLW - 1), rg2 = hw / DS_BLW, q2 = hw - rg2 * DS_BLW;
        uint32_t vi[NI], vb[NB];
        if (live) {
            const uint8_t* row0 = Pl + (long long)(y - 15) * stride + x - 15;
            if ((stride & 3) == 0) {  // every row has row 0's byte shift
                const uint8_t* c0 = reinterpret_cast<const uint8_t*>(
                    (reinterpret_cast<uintptr_t>(row0) & ~(uintptr_t)3) + 4 * (uintptr_t)q);
#pragma unroll
                for (int k = 0; k < NI; k++)
                    vi[k] = gfd::ldg(reinterpret_cast<const uint32_t*>(c0 + (long long)min(rg + 3 * k, DS_IC - 1) * stride));
            } else {
#pragma unroll
                for (int k = 0; k < NI; k++) {
                    const uintptr_t a = (uintptr_t)(row0 + (long long)min(rg + 3 * k, DS_IC - 1) * stride);
                    vi[k] = gfd::ldg(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3) + q);
                }
            }
        }
        if (win) {  // blurred rows pitched to 64 B: one byte shift for the window
            const uint32_t* c0 = reinterpret_cast<const uint32_t*>(
                                     reinterpret_cast<uintptr_t>(B + (long long)(y - 18) * pwl + x - 18) & ~(uintptr_t)3) +
                                 q2;
#pragma unroll
            for (int k = 0; k < NB; k++) vb[k] = gfd::ldg(c0 + (long long)min(rg2 + 3 * k, DS_BL - 1) * (pwl >> 2));
        }
        if (live) {
#pragma unroll
            for (int k = 0; k < NI; k++) W.ic[min(rg + 3 * k, DS_IC - 1) * DS_ICW + q] = vi[k];
        }
        if (win) {
#pragma unroll
            for (int k = 0; k < NB; k++) W.bl[min(rg2 + 3 * k, DS_BL - 1) * DS_BLW + q2] = vb[k];
        }
        if (hl < DS_IC) W.ic_sh[hl] = (uint8_t)((uintptr_t)(Pl + (long long)(y - 15 + hl) * stride + x - 15) & 3);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const uint8_t* bl8 = reinterpret_cast<const uint8_t*>(W.bl);

    // IC_Angle: 31 pixels of the 31x31 square per lane (row hl); pixels outside
    // the circular patch (|u| > umax[|v|]) weigh 0. Integer moments: order-free.
    // The row's 31 bytes realigned to 8 dwords; sum p and sum (u + 15) p over
    // the patch as v_dot4_u32_u8 against the row's weight dwords (exact), then
    // m10 = sum (u + 15) p - 15 sum p.
    int m10 = 0, m01 = 0;
    if (hl < 31) {
        const int v = hl - 15, av = v < 0 ? -v : v;
        const uint32_t* row = W.ic + hl * DS_ICW;
        const uint32_t sh = W.ic_sh[hl];
        uint32_t s1 = 0, s0 = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t px = __builtin_amdgcn_alignbyte(row[j + 1], row[j], sh);
            s1 = __builtin_amdgcn_udot4(px, sh_ictab[av * 8 + j], s1, false);
            s0 = __builtin_amdgcn_udot4(px, sh_ictab[128 + av * 8 + j], s0, false);
        }
        m10 = (int)s1 - 15 * (int)s0;
        m01 = v * (int)s0;
    }
    m10 = half_sum(m10);
    m01 = half_sum(m01);
    const float angle = fast_atan2f((float)m01, (float)m10);

    // rBRIEF: lane hl of the half computes descriptor byte hl (16 tests). The
    // blurred rows are pitched to 64 B, so every window row has the same byte
    // shift in its first dword.
    const int bsh = (int)((uintptr_t)(B + (long long)(y - 18) * pwl + x - 18) & 3);
    {
        const float factorPI = (float)(M_PI / 180.f);
        const float ang = angle * factorPI;
        const float a = gflibm::cosf(ang), b = gflibm::sinf(ang);  // glibc cosf/sinf (ORBextractor.cc:167)
        int val = 0;
        // the two sample sources in separate loops (a half's keypoint is
        // either inside or near the border), so the window's loop keeps its
        // LDS base and the rotation in registers across the 16 tests
        auto rot = [&](int bit, int q, int& rx, int& ry) {
            const uint32_t pt = sh_pat[bit * 32 + hl] >> (16 * q);
            const float px = (float)(int8_t)(pt & 0xff), py = (float)(int8_t)((pt >> 8) & 0xff);
            ry = __float2int_rn(px * b + py * a);
            rx = __float2int_rn(px * a - py * b);
        };
        if (win) {
            const uint8_t* ctr = bl8 + bsh + 18 * (4 * DS_BLW) + 18;  // the keypoint's byte in the window
#pragma unroll
            for (int bit = 0; bit < 8; bit++) {
                int t[2];
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    int rx, ry;
                    rot(bit, q, rx, ry);
#if DESC_B64
                    const int a8 = (int)(ctr - reinterpret_cast<const uint8_t*>(W.bl)) + ry * (4 * DS_BLW) + rx;
                    const uint64_t w8 = *reinterpret_cast<const uint64_t*>(bl8 + (a8 & ~7));
                    t[q] = (int)((w8 >> (8 * (a8 & 7))) & 0xffu);
#else
                    t[q] = ctr[ry * (4 * DS_BLW) + rx];
#endif
                }
                val |= (t[0] < t[1]) << bit;
            }
        } else if (live) {
#pragma unroll
            for (int bit = 0; bit < 8; bit++) {
                int t[2];
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    int rx, ry;
                    rot(bit, q, rx, ry);
                    const int xx = x + rx, yy = y + ry;
                    const bool inside = xx >= 0 && xx < w && yy >= 0 && yy < h;
                    t[q] = inside ? B[(long long)yy * pwl + xx]
                                  : gfd::ldg(Pl + (long long)gfd::reflect101(yy, h) * stride + gfd::reflect101(xx, w));
                }
                val |= (t[0] < t[1]) << bit;
            }
        }
        if (live) desc[((long long)f * cap + k) * 32 + hl] = (uint8_t)val;
    }
    if (live && hl == 0) {
        gf_keypoint kp;
        const float s = g.scale[l];
        kp.x = l ? (float)x * s : (float)x;
        kp.y = l ? (float)y * s : (float)y;
        kp.size = (float)(int)(31 * s);
        kp.angle = angle;
        kp.response = Ent<E>::response(e);
        kp.octave = l;
        kp.class_id = -1;
        kps[(long long)f * cap + k] = kp;
    }
}

}  // namespace

// ====================================================================== host
struct gf_extractor {
    gf_ctx* ctx = nullptr;
    hipEvent_t stage_ev = nullptr;  // gf::extract_stage_event
    int stage_after = -1;
    int nfeatures = 0, nlevels = 0, fast_th = 20, min_th = 7, width = 0, height = 0, max_batch = 0;
    bool harris = false;  // scoreType HARRIS_SCORE (0): u64 list entries carrying the Harris response
    float scale_factor = 1.2f;
    LevelGeom g{};
    std::vector<CellInfo> cells;
    std::vector<int> feat_per_level;
    int capacity = 0;
    long long list_stride = 0, lvl_stride = 0;
    size_t fast_lds = 0;
    size_t band_lds = 0;           // k_fast_cells_band's LDS (0: no large cell)
    std::vector<int> band_cells;   // cells whose window takes the banded kernel
    int* d_band = nullptr;
    int max_tiles = 0;
    // device buffers
    uint8_t *d_pyr = nullptr, *d_blur = nullptr, *d_score = nullptr;
    uint32_t *d_xtab = nullptr, *d_ytab = nullptr;  // k_pyramid's block-column / block-row records
    PyrGeom pg{};
    size_t pyr_lds = 0;
    int sel_maxnc = 0;  // most cells of a level (k_select's per-cell arrays)
    int pyr_g = PYR_G;  // k_pyramid's columns per item (1 when a 4-column group's taps span more than 7 bytes)
    CellInfo* d_cells = nullptr;
    void *d_lists = nullptr, *d_lvl = nullptr;  // uint32_t (FAST) or uint64_t (Harris) entries
    int *d_counts = nullptr, *d_lvl_counts = nullptr;
    // host-family staging
    uint8_t* d_img = nullptr;
    gf_keypoint* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int* d_nout = nullptr;
    // last batch (debug hook)
    Planes last{};
};

static int cv_round_f(float v) { return (int)std::lrintf(v); }
static int cv_floor_f(float v) {
    int i = (int)v;
    return i - (i > v);
}

// k_fast_cells keeps a cell's whole window (score rows, retry ROI, survivor
// bits) in LDS up to FC_LDS_MAX bytes; larger windows (small nFeatures) run
// k_fast_cells_band within FC_BAND_LDS.
constexpr size_t FC_LDS_MAX = 64 * 1024, FC_BAND_LDS = 120 * 1024;

static int plan_extractor(gf_extractor* ex) {
    const int nl = ex->nlevels;
    LevelGeom& g = ex->g;
    memset(&g, 0, sizeof(g));
    g.nlevels = nl;
    // ORBextractor::ORBextractor (:464-494): scale tables and level quotas.
    const double sf = ex->scale_factor;
    std::vector<float> scale(nl), inv(nl);
    scale[0] = 1.f;
    for (int i = 1; i < nl; i++) scale[i] = (float)((double)scale[i - 1] * sf);
    float invs = (float)(1.0f / sf);
    inv[0] = 1.f;
    for (int i = 1; i < nl; i++) inv[i] = inv[i - 1] * invs;
    ex->feat_per_level.assign(nl, 0);
    float factor = (float)(1.0 / sf);
    float nd = ex->nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
    int sum = 0;
    for (int l = 0; l < nl - 1; l++) {
        ex->feat_per_level[l] = cv_round_f(nd);
        sum += ex->feat_per_level[l];
        nd *= factor;
    }
    ex->feat_per_level[nl - 1] = std::max(ex->nfeatures - sum, 0);

    long long off = 0, boff = 0;
    for (int l = 0; l < nl; l++) {
        g.w[l] = cv_round_f((float)ex->width * inv[l]);
        g.h[l] = cv_round_f((float)ex->height * inv[l]);
        g.pw[l] = (g.w[l] + 63) & ~63;
        g.scale[l] = scale[l];
        GF_CHECK(g.w[l] >= 40 && g.h[l] >= 40 && g.w[l] < 4096 && g.h[l] < 4096, GF_ERR_ARG,
                 "level size out of supported range");
        if (l > 0) {
            g.off[l] = off;
            off += ((long long)g.pw[l] * g.h[l] + 255) & ~255LL;
        }
        g.boff[l] = boff;
        boff += ((long long)g.pw[l] * g.h[l] + 255) & ~255LL;
    }
    g.slab = off;
    g.bslab = boff;
    // blur tiles
    int t = 0;
    for (int l = 0; l < nl; l++) {
        g.tile_begin[l] = t;
        g.tiles_x[l] = (g.w[l] + BT_W - 1) / BT_W;
        t += g.tiles_x[l] * ((g.h[l] + BT_H - 1) / BT_H);
    }
    g.tile_begin[nl] = t;
    ex->max_tiles = t;

    // ComputeKeyPoints cell grids (:540-618).
    ex->cells.clear();
    ex->sel_maxnc = 0;
    ex->band_cells.clear();
    ex->band_lds = 0;
    long long cap_off = 0, lvl_off = 0;
    size_t max_lds = 0;
    const float imageRatio = (float)g.w[0] / g.h[0];
    for (int l = 0; l < nl; l++) {
        const int nDesired = ex->feat_per_level[l];
        const int levelCols = (int)std::sqrt((float)nDesired / (5 * imageRatio));
        const int levelRows = (int)(imageRatio * levelCols);
        GF_CHECK(levelCols > 0 && levelRows > 0, GF_ERR_UNSUPPORTED, "level with an empty cell grid");
        const int minB = 16, maxBX = g.w[l] - 16, maxBY = g.h[l] - 16;
        const int W = maxBX - minB, H = maxBY - minB;
        const int cellW = (int)std::ceil((float)W / levelCols);
        const int cellH = (int)std::ceil((float)H / levelRows);
        const int nCells = levelRows * levelCols;
        GF_CHECK(nCells <= SEL_MAX_CELLS, GF_ERR_UNSUPPORTED, "too many cells per level");
        ex->sel_maxnc = std::max(ex->sel_maxnc, nCells);
        g.nfcell[l] = (int)std::ceil((float)nDesired / nCells);
        g.ndesired[l] = nDesired;
        g.cell_begin[l] = (int)ex->cells.size();
        g.lvl_off[l] = lvl_off;
        std::vector<int> iniXCol(levelCols, 0);
        float hY = cellH + 6;
        long long lvl_cap = 0;
        for (int i = 0; i < levelRows; i++) {
            const float iniY = minB + i * cellH - 3;
            bool rowSkip = false;
            if (i == levelRows - 1) {
                hY = maxBY + 3 - iniY;
                if (hY <= 0) rowSkip = true;
            }
            float hX = cellW + 6;
            for (int j = 0; j < levelCols; j++) {
                float iniX;
                if (i == 0) {
                    iniX = minB + j * cellW - 3;
                    iniXCol[j] = (int)iniX;
                } else
                    iniX = iniXCol[j];
                CellInfo ci{};
                ci.level = l;
                ci.valid = 0;
                if (!rowSkip) {
                    bool skip = false;
                    if (j == levelCols - 1) {
                        hX = maxBX + 3 - iniX;
                        if (hX <= 0) skip = true;
                    }
                    if (!skip) {
                        ci.x0 = (int)iniX;
                        ci.y0 = (int)iniY;
                        ci.w = (int)hX;
                        ci.h = (int)hY;
                        // a degenerate ROI (< 7 px) is processed and detects nothing, as FAST does
                        ci.valid = 1;
                        int dw = std::max(ci.w - 6, 0), dh = std::max(ci.h - 6, 0);
                        ci.cap = ((dw + 1) / 2) * ((dh + 1) / 2);
                        ci.cap_off = cap_off;
                        cap_off += ci.cap;
                        lvl_cap += ci.cap;
                        const size_t pitch = 4 * (size_t)((dw + 6) / 4), bits = 16 * (((size_t)dw * dh + 127) / 128);
                        const FcLayout fl = fc_layout(dw, dh, ci.w, ci.h);
                        const size_t lds = fl.total;
                        if (lds <= FC_LDS_MAX && fl.ndw <= FC_NT) {
                            max_lds = std::max(max_lds, lds);
                        } else {  // k_fast_cells_band: bands of BH rows (halo rows, ROI rows of the retry)
                            auto band_lds = [&](size_t bh) {
                                return bits + (bh + 3) * pitch + ((bh + 3 + 15) & ~(size_t)15) + (bh + 8) * ci.w;
                            };
                            size_t bh = std::min<size_t>(dh, 64);
                            while (bh > 4 && band_lds(bh) > FC_BAND_LDS) bh /= 2;
                            GF_CHECK(band_lds(bh) <= FC_BAND_LDS, GF_ERR_UNSUPPORTED,
                                     "cell window too large even for the banded FAST kernel");
                            ci.band = (int)bh;
                            ex->band_cells.push_back((int)ex->cells.size());
                            ex->band_lds = std::max(ex->band_lds, band_lds(bh));
                        }
                        GF_CHECK(ci.x0 >= 0 && ci.y0 >= 0 && ci.x0 + ci.w <= g.w[l] && ci.y0 + ci.h <= g.h[l],
                                 GF_ERR_ARG, "cell ROI outside level");
                    }
                }
                ex->cells.push_back(ci);
            }
        }
        lvl_off += std::max(lvl_cap, (long long)nDesired);
    }
    g.cell_begin[nl] = (int)ex->cells.size();
    g.lvl_off[nl] = lvl_off;
    g.ncells = (int)ex->cells.size();
    ex->list_stride = cap_off;
    ex->lvl_stride = lvl_off;
    ex->fast_lds = max_lds;
    ex->capacity = 0;
    for (int l = 0; l < nl; l++) ex->capacity += ex->feat_per_level[l];
    return GF_OK;
}

static void resize_tables(int sw, int sh, int dw, int dh, std::vector<int2>& xt, std::vector<int2>& yt) {
    // cv::resize INTER_LINEAR coefficient set-up (fixed point, 2048 = 1.0).
    const int ONE = 2048;
    double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    xt.resize(dw);
    yt.resize(dh);
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor_f(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx >= sw - 1) fx = 0, sx = sw - 1;
        int a0 = (short)cv_round_f((1.f - fx) * ONE), a1 = (short)cv_round_f(fx * ONE);
        xt[dx] = make_int2(sx, (a0 & 0xffff) | (a1 << 16));
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor_f(fy);
        fy -= sy;
        int b0 = (short)cv_round_f((1.f - fy) * ONE), b1 = (short)cv_round_f(fy * ONE);
        yt[dy] = make_int2(sy, (b0 & 0xffff) | (b1 << 16));
    }
}

// k_pyramid's blocks: each level cut into the same nbx x nby grid; top-down
// from the last level, a block's required span at level l is its owned
// pixels plus the source pixels (both taps) of its required span at l + 1
// (level 0: the source pixels only). Blocks start near 128 x 96 level-0 px
// and shrink until every computed span is at most 256 columns and the
// two LDS buffers (even / odd levels) fit 64 KB.
static void pyr_axis(const LevelGeom& g, const std::vector<std::vector<int2>>& tabs, bool is_x, int nb,
                     std::vector<PyrSpan>& out, int& maxspan) {
    const int nl = g.nlevels;
    out.assign((size_t)nl * nb, PyrSpan{});
    maxspan = 0;
    for (int k = 0; k < nb; k++) {
        int lo = 0, hi = 0;
        for (int l = nl - 1; l >= 0; l--) {
            const int n = is_x ? g.w[l] : g.h[l];
            int rlo = 0, rhi = 0;
            if (l < nl - 1) {  // the taps of level l + 1's required span (rows clamped as the kernel clamps them)
                const std::vector<int2>& t = tabs[l + 1];
                rlo = std::min(std::max(t[lo].x, 0), n - 1);
                rhi = std::min(std::max(t[hi].x + 1, 0), n - 1);
            }
            PyrSpan s{};
            if (l >= 1) {
                // columns: block boundaries and required spans start at multiples
                // of 4, so k_pyramid's 4-column groups store aligned dwords
                const int al = is_x ? 4 : 1;
                auto bound = [&](int kk) {
                    return kk >= nb ? n : (int)((long long)kk * n / nb) / al * al;
                };
                const int olo = bound(k), ohi = bound(k + 1);
                s.olo = (int16_t)olo;
                s.ohi = (int16_t)ohi;
                lo = (l < nl - 1 ? std::min(rlo, olo) : olo) / al * al;
                hi = l < nl - 1 ? std::max(rhi, ohi - 1) : ohi - 1;
                maxspan = std::max(maxspan, hi - lo + 1);
            } else {
                lo = rlo;
                hi = rhi;
            }
            s.lo = (int16_t)lo;
            s.hi = (int16_t)hi;
            out[(size_t)l * nb + k] = s;
        }
    }
}

static bool pyr_plan(const LevelGeom& g, const std::vector<std::vector<int2>>& xts,
                     const std::vector<std::vector<int2>>& yts, PyrGeom& pg, std::vector<PyrSpan>& spx,
                     std::vector<PyrSpan>& spy, size_t& lds) {
    const int nl = g.nlevels;
    int nbx = std::max(1, (g.w[0] + 127) / 128), nby = std::max(1, (g.h[0] + 95) / 96);
    const int nmax = std::min(g.w[nl - 1], g.h[nl - 1]) / 2;  // at least two owned pixels per block and level
    while (nbx <= nmax && nby <= nmax) {
        int mx, my;
        pyr_axis(g, xts, true, nbx, spx, mx);
        pyr_axis(g, yts, false, nby, spy, my);
        size_t buf[2] = {0, 0};
        for (int l = 0; l < nl; l++)
            for (int kx = 0; kx < nbx; kx++)
                for (int ky = 0; ky < nby; ky++) {
                    const PyrSpan& a = spx[(size_t)l * nbx + kx];
                    const PyrSpan& b = spy[(size_t)l * nby + ky];
                    const size_t pitch = (size_t)((a.hi - a.lo + 1 + 8 + 3) & ~3);
                    buf[l & 1] = std::max(buf[l & 1], pitch * (size_t)(b.hi - b.lo + 1));
                }
        buf[0] = (buf[0] + 15) & ~(size_t)15;
        if (mx <= 256 && buf[0] + buf[1] <= 64 * 1024) {
            pg.nbx = nbx;
            pg.nby = nby;
            pg.lds_a = (int)buf[0];
            lds = buf[0] + buf[1];
            return true;
        }
        if (mx > 256 || (double)g.w[0] / nbx >= (double)g.h[0] / nby) nbx++;
        else nby++;
    }
    return false;
}

static void free_extractor(gf_extractor* ex) {
    (void)hipFree(ex->d_pyr);
    (void)hipFree(ex->d_blur);
    (void)hipFree(ex->d_score);
    (void)hipFree(ex->d_xtab);
    (void)hipFree(ex->d_ytab);
    (void)hipFree(ex->d_cells);
    (void)hipFree(ex->d_band);
    (void)hipFree(ex->d_lists);
    (void)hipFree(ex->d_lvl);
    (void)hipFree(ex->d_counts);
    (void)hipFree(ex->d_lvl_counts);
    (void)hipFree(ex->d_img);
    (void)hipFree(ex->d_kps);
    (void)hipFree(ex->d_desc);
    (void)hipFree(ex->d_nout);
}

static int upload_constants(int device) {
    static unsigned long long done_mask = 0;
    if (done_mask & (1ull << device)) return GF_OK;
    {
        uint32_t p8[256];
        for (int i = 0; i < 256; i++) {
            uint32_t v = 0;
            for (int j = 0; j < 4; j++) {
                const int c = kOrbPattern31[4 * i + j];
                GF_CHECK(c >= -128 && c <= 127, GF_ERR_ARG, "pattern coordinate out of int8 range");
                v |= (uint32_t)(uint8_t)(int8_t)c << (8 * j);
            }
            p8[i] = v;
        }
        GF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern8), p8, sizeof(p8)));
    }
    // umax of the circular patch (ORBextractor.cc:500-517)
    int umax[16];
    const int hp = 15;
    int vmax = cv_floor_f(hp * std::sqrt(2.f) / 2 + 1);
    float vminf = hp * std::sqrt(2.f) / 2;
    int vmin = (int)vminf + ((int)vminf < vminf);
    const double hp2 = hp * hp;
    for (int v = 0; v <= vmax; ++v) umax[v] = (int)std::lrint(std::sqrt(hp2 - v * v));
    for (int v = hp, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
    {
        uint32_t tab[256] = {};
        for (int av = 0; av < 16; av++)
            for (int c = 0; c < 31; c++) {
                const int u = c - 15;
                if (u < -umax[av] || u > umax[av]) continue;
                tab[av * 8 + c / 4] |= (uint32_t)(u + 15) << (8 * (c % 4));
                tab[128 + av * 8 + c / 4] |= 1u << (8 * (c % 4));
            }
        GF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_ic_tab), tab, sizeof(tab)));
    }
    done_mask |= 1ull << device;
    return GF_OK;
}

static int extract_planes(gf_extractor* ex, int nframes, Planes P, gf_keypoint* d_kps, uint8_t* d_desc,
                          int32_t* d_counts, int cap, void* stream);
template <typename E>
static int select_describe(gf_extractor* ex, int nframes, Planes P, gf_keypoint* d_kps, uint8_t* d_desc,
                           int32_t* d_counts, int cap, hipStream_t s);

extern "C" {

int gf_extractor_create(gf_ctx* ctx, int nfeatures, float scale_factor, int nlevels, int score_type, int fast_th,
                        int width, int height, int max_batch, gf_extractor** out) {
    GF_CHECK(ctx && out, GF_ERR_ARG, "null arg");
    GF_CHECK(score_type == 0 || score_type == 1, GF_ERR_ARG, "scoreType: 0 HARRIS_SCORE, 1 FAST_SCORE");
    GF_CHECK(nlevels >= 1 && nlevels <= GF_MAX_LEVELS, GF_ERR_ARG, "nlevels out of range");
    GF_CHECK(nfeatures > 0 && scale_factor > 1.f && width > 0 && height > 0 && max_batch > 0, GF_ERR_ARG,
             "bad extractor parameters");
    GF_CHECK(fast_th >= 0 && fast_th < 255, GF_ERR_ARG, "bad FAST threshold");
    GF_HIP(hipSetDevice(ctx->device));
    int rc = upload_constants(ctx->device);
    if (rc) return rc;
    gf_extractor* ex = new gf_extractor();
    ex->ctx = ctx;
    ex->nfeatures = nfeatures;
    ex->scale_factor = scale_factor;
    ex->nlevels = nlevels;
    ex->fast_th = fast_th;
    ex->width = width;
    ex->height = height;
    ex->max_batch = max_batch;
    ex->harris = score_type == 0;
    rc = plan_extractor(ex);
    if (rc) {
        delete ex;
        return rc;
    }
    const LevelGeom& g = ex->g;
    auto cleanup = [&](hipError_t e) {
        free_extractor(ex);
        delete ex;
        return gf::fail(GF_ERR_HIP, std::string("extractor alloc: ") + hipGetErrorString(e));
    };
    hipError_t e;
#define ALLOC(p, bytes)                              \
    if ((e = hipMalloc((void**)&(p), (bytes))) != hipSuccess) return cleanup(e);
    ALLOC(ex->d_pyr, std::max<long long>(g.slab, 256) * max_batch);
    ALLOC(ex->d_blur, g.bslab * max_batch);
    ALLOC(ex->d_score, g.bslab * max_batch);
    ALLOC(ex->d_cells, sizeof(CellInfo) * ex->cells.size());
    const size_t esz = ex->harris ? sizeof(uint64_t) : sizeof(uint32_t);
    ALLOC(ex->d_lists, esz * ex->list_stride * max_batch);
    ALLOC(ex->d_lvl, esz * ex->lvl_stride * max_batch);
    ALLOC(ex->d_band, sizeof(int) * std::max<size_t>(ex->band_cells.size(), 1));
    ALLOC(ex->d_counts, sizeof(int) * g.ncells * max_batch);
    ALLOC(ex->d_lvl_counts, sizeof(int) * nlevels * max_batch);
    ALLOC(ex->d_img, (size_t)width * height);
    ALLOC(ex->d_kps, sizeof(gf_keypoint) * ex->capacity);
    ALLOC(ex->d_desc, 32 * (size_t)ex->capacity);
    ALLOC(ex->d_nout, sizeof(int));
    // resize tables for levels 1..nl-1, and k_pyramid's block spans
    std::vector<std::vector<int2>> xts(nlevels), yts(nlevels);
    for (int l = 1; l < nlevels; l++) resize_tables(g.w[l - 1], g.h[l - 1], g.w[l], g.h[l], xts[l], yts[l]);
    std::vector<PyrSpan> spx, spy;
    if (nlevels > 1 && !pyr_plan(g, xts, yts, ex->pg, spx, spy, ex->pyr_lds)) {
        free_extractor(ex);
        delete ex;
        return gf::fail(GF_ERR_UNSUPPORTED, "scale factor too large for the pyramid blocks");
    }
    // k_pyramid's column groups: PYR_G columns whose taps lie within 8 bytes
    // of the group's first tap (else one column per item)
    for (int l = 1; l < nlevels && ex->pyr_g > 1; l++)
        for (int k = 0; k < ex->pg.nbx; k++) {
            const PyrSpan& sp = spx[(size_t)l * ex->pg.nbx + k];
            for (int x0 = sp.lo; x0 <= sp.hi; x0 += PYR_G)
                if (xts[l][std::min(x0 + PYR_G - 1, (int)sp.hi)].x - xts[l][x0].x + 1 > 7) ex->pyr_g = 1;
        }
    // the block-column / block-row records (k_pyramid)
    std::vector<uint32_t> xrec, yrec;
    if (nlevels > 1) {
        const int G = ex->pyr_g;
        auto pack = [](const std::vector<std::vector<uint32_t>>& r, std::vector<uint32_t>& rec) -> int {
            size_t stride = 0;
            for (const auto& v : r) stride = std::max(stride, v.size());
            stride = (stride + 3) & ~(size_t)3;
            rec.assign(stride * r.size(), 0u);
            for (size_t k = 0; k < r.size(); k++) std::copy(r[k].begin(), r[k].end(), rec.begin() + k * stride);
            return (int)stride;
        };
        auto head = [&](std::vector<uint32_t>& v, const std::vector<PyrSpan>& sp, int nb, int k) {
            for (int l = 0; l < nlevels; l++) {
                const uint2 u = __builtin_bit_cast(uint2, sp[(size_t)l * nb + k]);
                v.push_back(u.x);
                v.push_back(u.y);
            }
        };
        bool ok = true;
        std::vector<std::vector<uint32_t>> rx(ex->pg.nbx), ry(ex->pg.nby);
        for (int k = 0; k < ex->pg.nbx; k++) {
            head(rx[k], spx, ex->pg.nbx, k);
            for (int l = 1; l < nlevels; l++) {
                const PyrSpan& s = spx[(size_t)l * ex->pg.nbx + k];
                const PyrSpan& ss = spx[(size_t)(l - 1) * ex->pg.nbx + k];
                for (int x0 = s.lo; x0 <= s.hi; x0 += G) {
                    const int c0 = xts[l][x0].x - ss.lo;
                    uint32_t h = (uint32_t)c0, own = 0;
                    std::vector<uint32_t> w;
                    for (int j = 0; j < G; j++) {
                        const int x = x0 + j;
                        if (x > s.hi) {  // past the span: weight 0; past the level's last column the
                            w.push_back(0u);  // byte lands in the row padding, stored with its group
                            own |= (uint32_t)(x >= g.w[l] && s.ohi == g.w[l]) << j;
                            continue;
                        }
                        const int d = xts[l][x].x - ss.lo - c0;
                        ok = ok && d >= 0 && d <= 6 && c0 >= 0 && c0 < 0x10000;
                        if (j) h |= (uint32_t)d << (12 + 4 * j);
                        own |= (uint32_t)(x >= s.olo && x < s.ohi) << j;
                        const uint32_t a = (uint32_t)xts[l][x].y;
                        ok = ok && (a & 0xffffu) + (a >> 16) <= 2049;
                        w.push_back(a);
                    }
                    rx[k].push_back(h | own << 28);
                    rx[k].insert(rx[k].end(), w.begin(), w.end());
                }
            }
        }
        for (int k = 0; k < ex->pg.nby; k++) {
            head(ry[k], spy, ex->pg.nby, k);
            for (int l = 1; l < nlevels; l++) {
                const PyrSpan& s = spy[(size_t)l * ex->pg.nby + k];
                const PyrSpan& ss = spy[(size_t)(l - 1) * ex->pg.nby + k];
                const int sh = g.h[l - 1];
                for (int y = s.lo; y <= s.hi; y++) {
                    const int r0 = std::min(std::max(yts[l][y].x, 0), sh - 1) - ss.lo;
                    const int r1 = std::min(std::max(yts[l][y].x + 1, 0), sh - 1) - ss.lo;
                    ok = ok && r0 >= 0 && r1 >= 0 && r0 < 0x8000 && r1 < 0x8000;
                    const uint32_t b = (uint32_t)yts[l][y].y;
                    ok = ok && (b & 0xffffu) + (b >> 16) <= 2049;
                    ry[k].push_back((uint32_t)r0 | (uint32_t)r1 << 16 | (uint32_t)(y >= s.olo && y < s.ohi) << 31);
                    ry[k].push_back(b);
                }
            }
        }
        if (!ok) {
            free_extractor(ex);
            delete ex;
            return gf::fail(GF_ERR_UNSUPPORTED, "pyramid tables outside the k_pyramid record ranges");
        }
        ex->pg.rx = pack(rx, xrec);
        ex->pg.ry = pack(ry, yrec);
        ex->pg.lds_img = (int)((ex->pyr_lds + 15) & ~(size_t)15);
        ex->pyr_lds = ex->pg.lds_img + sizeof(uint32_t) * (size_t)(ex->pg.rx + ex->pg.ry);
    }
    ALLOC(ex->d_xtab, sizeof(uint32_t) * std::max<size_t>(xrec.size(), 1));
    ALLOC(ex->d_ytab, sizeof(uint32_t) * std::max<size_t>(yrec.size(), 1));
#undef ALLOC
    if (!xrec.empty()) {
        GF_HIP(hipMemcpy(ex->d_xtab, xrec.data(), sizeof(uint32_t) * xrec.size(), hipMemcpyHostToDevice));
        GF_HIP(hipMemcpy(ex->d_ytab, yrec.data(), sizeof(uint32_t) * yrec.size(), hipMemcpyHostToDevice));
        GF_HIP(hipFuncSetAttribute((const void*)k_pyramid<PYR_G>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)ex->pyr_lds));
        GF_HIP(hipFuncSetAttribute((const void*)k_pyramid<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)ex->pyr_lds));
    }
    GF_HIP(hipMemcpy(ex->d_cells, ex->cells.data(), sizeof(CellInfo) * ex->cells.size(), hipMemcpyHostToDevice));
    if (!ex->band_cells.empty())
        GF_HIP(hipMemcpy(ex->d_band, ex->band_cells.data(), sizeof(int) * ex->band_cells.size(),
                         hipMemcpyHostToDevice));
    if (ex->harris) {
        GF_HIP(hipFuncSetAttribute((const void*)k_select_cells<uint64_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(SEL_CW * sel_cell_wave_lds<uint64_t>(ex->sel_maxnc))));
        GF_HIP(hipFuncSetAttribute((const void*)k_fast_cells<uint64_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)ex->fast_lds));
        GF_HIP(hipFuncSetAttribute((const void*)k_fast_cells_band<uint64_t>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)ex->band_lds));
    } else {
        GF_HIP(hipFuncSetAttribute((const void*)k_select_cells<uint32_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(SEL_CW * sel_cell_wave_lds<uint32_t>(ex->sel_maxnc))));
        GF_HIP(hipFuncSetAttribute((const void*)k_fast_cells<uint32_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)ex->fast_lds));
        GF_HIP(hipFuncSetAttribute((const void*)k_fast_cells_band<uint32_t>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)ex->band_lds));
    }
    *out = ex;
    return GF_OK;
}

int gf_extractor_destroy(gf_extractor* ex) {
    if (!ex) return GF_OK;
    (void)hipSetDevice(ex->ctx->device);
    free_extractor(ex);
    delete ex;
    return GF_OK;
}

int gf_extractor_info(gf_extractor* ex, int* nlevels, float* scale_factor, int* features_per_level) {
    GF_CHECK(ex, GF_ERR_ARG, "null extractor");
    if (nlevels) *nlevels = ex->nlevels;
    if (scale_factor) *scale_factor = ex->scale_factor;
    if (features_per_level)
        for (int l = 0; l < ex->nlevels; l++) features_per_level[l] = ex->feat_per_level[l];
    return GF_OK;
}

int gf_extractor_capacity(gf_extractor* ex, int* cap) {
    GF_CHECK(ex && cap, GF_ERR_ARG, "null arg");
    *cap = ex->capacity;
    return GF_OK;
}

int gf_orb_extract_batch_dev(gf_extractor* ex, int nframes, const uint8_t* d_imgs, size_t frame_stride, int stride,
                             gf_keypoint* d_kps, uint8_t* d_desc, int32_t* d_counts, int cap, void* stream) {
    GF_CHECK(ex && d_imgs && d_kps && d_desc && d_counts, GF_ERR_ARG, "null arg");
    Planes P{d_imgs, (long long)frame_stride, stride, nullptr, ex->d_pyr, ex->d_blur};
    return extract_planes(ex, nframes, P, d_kps, d_desc, d_counts, cap, stream);
}

int gf_orb_extract_ptrs_dev(gf_extractor* ex, int nframes, const uint8_t* const* d_img_ptrs, int stride,
                            gf_keypoint* d_kps, uint8_t* d_desc, int32_t* d_counts, int cap, void* stream) {
    GF_CHECK(ex && d_img_ptrs && d_kps && d_desc && d_counts, GF_ERR_ARG, "null arg");
    Planes P{nullptr, 0, stride, d_img_ptrs, ex->d_pyr, ex->d_blur};
    return extract_planes(ex, nframes, P, d_kps, d_desc, d_counts, cap, stream);
}

}  // extern "C"

static int extract_planes(gf_extractor* ex, int nframes, Planes P, gf_keypoint* d_kps, uint8_t* d_desc,
                          int32_t* d_counts, int cap, void* stream) {
    const int stride = P.stride0;
    GF_CHECK(nframes >= 0 && nframes <= ex->max_batch, GF_ERR_ARG, "nframes exceeds max_batch");
    GF_CHECK(cap >= ex->capacity, GF_ERR_CAP, "cap below extractor capacity");
    GF_CHECK(stride >= ex->width, GF_ERR_ARG,
             "row stride " + std::to_string(stride) + " below width " + std::to_string(ex->width));
    if (nframes == 0) return GF_OK;
    hipStream_t s = (hipStream_t)stream;
    const LevelGeom& g = ex->g;
    ex->last = P;
    gf_ctx* ctx = ex->ctx;
    {
        GF_PROF(ctx, s, "k_pyramid");
        if (ex->nlevels > 1)
        {
            if (ex->pyr_g == PYR_G)
                GF_LAUNCH(k_pyramid<PYR_G>, dim3(ex->pg.nbx * ex->pg.nby, nframes), PYR_NT, ex->pyr_lds, s, P, g,
                          ex->pg, ex->d_xtab, ex->d_ytab);
            else
                GF_LAUNCH(k_pyramid<1>, dim3(ex->pg.nbx * ex->pg.nby, nframes), PYR_NT, ex->pyr_lds, s, P, g, ex->pg,
                          ex->d_xtab, ex->d_ytab);
        }
    }
    if (ex->stage_ev && ex->stage_after == 0) GF_HIP(hipEventRecord(ex->stage_ev, s));
    {
        GF_PROF(ctx, s, "k_blur_fast");
        GF_LAUNCH(k_blur_fast, dim3(ex->max_tiles, nframes), 256, 0, s, P, g, ex->d_score, ex->fast_th);
    }
    if (ex->stage_ev && ex->stage_after == 1) GF_HIP(hipEventRecord(ex->stage_ev, s));
    return ex->harris ? select_describe<uint64_t>(ex, nframes, P, d_kps, d_desc, d_counts, cap, s)
                      : select_describe<uint32_t>(ex, nframes, P, d_kps, d_desc, d_counts, cap, s);
}

// k_fast_cells (+ k_fast_cells_band), k_select, k_describe on list entries E.
template <typename E>
static int select_describe(gf_extractor* ex, int nframes, Planes P, gf_keypoint* d_kps, uint8_t* d_desc,
                           int32_t* d_counts, int cap, hipStream_t s) {
    const LevelGeom& g = ex->g;
    gf_ctx* ctx = ex->ctx;
    E* lists = reinterpret_cast<E*>(ex->d_lists);
    E* lvl = reinterpret_cast<E*>(ex->d_lvl);
    {
        GF_PROF(ctx, s, "k_fast_cells");
        GF_LAUNCH(k_fast_cells<E>, dim3(g.ncells, nframes), FC_NT, ex->fast_lds, s, P, g, ex->d_score, ex->d_cells,
                  lists, ex->list_stride, ex->d_counts, ex->fast_th, ex->min_th);
        if (!ex->band_cells.empty())
            GF_LAUNCH(k_fast_cells_band<E>, dim3((int)ex->band_cells.size(), nframes), 256, ex->band_lds, s, P, g,
                      ex->d_score, ex->d_cells, ex->d_band, lists, ex->list_stride, ex->d_counts, ex->fast_th,
                      ex->min_th);
    }
    if (ex->stage_ev && ex->stage_after == 2) GF_HIP(hipEventRecord(ex->stage_ev, s));
    {
        GF_PROF(ctx, s, "k_select");
        GF_LAUNCH(k_select_cells<E>, dim3((g.ncells + SEL_CW - 1) / SEL_CW, nframes), 64 * SEL_CW,
                  SEL_CW * sel_cell_wave_lds<E>(ex->sel_maxnc), s, g, ex->d_cells, lists, ex->list_stride,
                  ex->d_counts, lvl, ex->lvl_stride, ex->d_lvl_counts, ex->sel_maxnc);
        GF_LAUNCH(k_select_level<E>, dim3(nframes, ex->nlevels), 64, sel_wave_bytes<E>(SEL_BUF), s, g, lvl,
                  ex->lvl_stride, ex->d_lvl_counts);
    }
    if (ex->stage_ev && ex->stage_after == 3) GF_HIP(hipEventRecord(ex->stage_ev, s));
    {
        GF_PROF(ctx, s, "k_describe");
        GF_LAUNCH(k_describe<E>, dim3((ex->capacity + 7) / 8, nframes), 256, 0, s, P, g, lvl, ex->lvl_stride,
                  ex->d_lvl_counts, d_kps, d_desc, d_counts, cap);
    }
    if (ex->stage_ev && ex->stage_after == 4) GF_HIP(hipEventRecord(ex->stage_ev, s));
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf::extract_stage_event(gf_extractor* ex, void* ev, int after) {
    GF_CHECK(ex, GF_ERR_ARG, "null extractor");
    GF_CHECK(!ev || (after >= 0 && after <= 4), GF_ERR_ARG, "extraction stage must be 0..4");
    ex->stage_ev = (hipEvent_t)ev;
    ex->stage_after = ev ? after : -1;
    return GF_OK;
}

extern "C" {

int gf_orb_extract(gf_extractor* ex, const uint8_t* img, int stride, gf_keypoint* kps, uint8_t* desc, int cap,
                   int* n_out) {
    GF_CHECK(ex && n_out, GF_ERR_ARG, "null arg");
    *n_out = 0;
    if (!img) return GF_OK;  // empty image (ORBextractor.cc:772)
    GF_CHECK(kps && desc, GF_ERR_ARG, "null output");
    GF_HIP(hipSetDevice(ex->ctx->device));
    hipStream_t s = ex->ctx->stream;
    GF_HIP(hipMemcpy2DAsync(ex->d_img, ex->width, img, stride, ex->width, ex->height, hipMemcpyHostToDevice, s));
    int rc = gf_orb_extract_batch_dev(ex, 1, ex->d_img, (size_t)ex->width * ex->height, ex->width, ex->d_kps,
                                      ex->d_desc, ex->d_nout, ex->capacity, s);
    if (rc) return rc;
    int n = 0;
    GF_HIP(hipMemcpyAsync(&n, ex->d_nout, sizeof(int), hipMemcpyDeviceToHost, s));
    GF_HIP(hipStreamSynchronize(s));
    *n_out = n;
    GF_CHECK(n <= cap, GF_ERR_CAP, "keypoint capacity too small");
    if (n) {
        GF_HIP(hipMemcpyAsync(kps, ex->d_kps, sizeof(gf_keypoint) * n, hipMemcpyDeviceToHost, s));
        GF_HIP(hipMemcpyAsync(desc, ex->d_desc, 32 * (size_t)n, hipMemcpyDeviceToHost, s));
        GF_HIP(hipStreamSynchronize(s));
    }
    return GF_OK;
}

#ifdef GF_SEL_STAMP
int gf_debug_sel_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sel_stamp), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sel_stamp), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

int gf_extractor_debug_level(gf_extractor* ex, int frame, int level, int which, uint8_t* out, int* w, int* h) {
    GF_CHECK(ex && w && h, GF_ERR_ARG, "null arg");
    GF_CHECK(level >= 0 && level < ex->nlevels && frame >= 0 && frame < ex->max_batch, GF_ERR_ARG, "bad index");
    const LevelGeom& g = ex->g;
    *w = g.w[level];
    *h = g.h[level];
    if (!out) return GF_OK;
    GF_HIP(hipSetDevice(ex->ctx->device));
    GF_HIP(hipStreamSynchronize(ex->ctx->stream));
    if (which == 1) {
        GF_HIP(hipMemcpy2D(out, g.w[level], ex->d_blur + (long long)frame * g.bslab + g.boff[level], g.pw[level],
                           g.w[level], g.h[level], hipMemcpyDeviceToHost));
    } else if (level == 0) {
        GF_CHECK(ex->last.img0 || ex->last.ptrs, GF_ERR_ARG, "no batch run yet");
        if (ex->last.ptrs) {
            const uint8_t* src = nullptr;
            GF_HIP(hipMemcpy(&src, ex->last.ptrs + frame, sizeof(src), hipMemcpyDeviceToHost));
            GF_HIP(hipMemcpy2D(out, g.w[0], src, ex->last.stride0, g.w[0], g.h[0], hipMemcpyDeviceToHost));
            return GF_OK;
        }
        GF_HIP(hipMemcpy2D(out, g.w[0], ex->last.img0 + (long long)frame * ex->last.fstride0, ex->last.stride0, g.w[0],
                           g.h[0], hipMemcpyDeviceToHost));
    } else {
        GF_HIP(hipMemcpy2D(out, g.w[level], ex->d_pyr + (long long)frame * g.slab + g.off[level], g.pw[level],
                           g.w[level], g.h[level], hipMemcpyDeviceToHost));
    }
    return GF_OK;
}

}  // extern "C"
