// Shared device pieces of the projection matchers (match.hip) and the active
// map matching of the good-feature module (gf.hip): frame constants, the
// 64x48 keypoint grid (Frame.cc:100-131, :300-377) and Hamming distance.
#pragma once
#include "common.h"

#define GRID_COLS 64
#define GRID_ROWS 48
#define NCELLS (GRID_COLS * GRID_ROWS)
#define KP_MAX 4096
#define Q_MAX 8192
#ifndef MATCH_THREADS
#define MATCH_THREADS 1024
#endif
#define TH_HIGH 100
#define HISTO_LENGTH 30


struct FrameConst {
    int min_x, max_x, min_y, max_y;
    float fx, fy, cx, cy;
    int nlevels;
    float invW, invH;
    float scales[16];
};


__device__ __forceinline__ int hamming32(const uint8_t* a, const uint8_t* b) {
    const uint4* pa = (const uint4*)a;
    const uint4* pb = (const uint4*)b;
    uint4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ int hamming_regs(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ void transform3(const float* T, const float* P, float* Pc) {
#pragma unroll
    for (int r = 0; r < 3; r++) {
        float a = T[4 * r + 0] * P[0];
        float b = T[4 * r + 1] * P[1];
        float c = T[4 * r + 2] * P[2];
        Pc[r] = ((a + b) + c) + T[4 * r + 3];
    }
}

__device__ __forceinline__ bool level_ok(int oct, int minL, int maxL) {
    const bool check = !(minL == -1 && maxL == -1);
    const bool same = check && minL == maxL;
    if (check && !same) return !(oct < minL || oct > maxL);
    if (same) return oct == minL;
    return true;
}

namespace gf {
FrameConst make_frame_const(const gf_frame_info* fi);
}

// Builds the grid CSR (cells ix-major, ascending keypoint index inside a cell)
// and loads the claim state; `scratch` (>= n ints) is clobbered. Must be
// called by all `nthreads` threads of the workgroup. The placement advances
// cell_start[c] itself to the cell's end, and a shift by one entry (top
// chunk first, so no entry is overwritten before it is read) turns the ends
// back into starts: no separate cursor array (12 KB of LDS fewer).
__device__ __forceinline__ void build_grid(const FrameConst& fc, const gf_keypoint* K, int n, const int32_t* kp2mp,
                                           int* cell_start, int* items, int* claim, int* scratch, int nthreads) {
    const int tid = threadIdx.x;
    for (int c = tid; c < NCELLS + 1; c += nthreads) cell_start[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += nthreads) {
        const gf_keypoint kp = K[i];
        int px = (int)roundf((kp.x - fc.min_x) * fc.invW);
        int py = (int)roundf((kp.y - fc.min_y) * fc.invH);
        int c = (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) ? -1 : px * GRID_ROWS + py;
        scratch[i] = c;
        if (c >= 0) atomicAdd(&cell_start[c + 1], 1);
        claim[i] = kp2mp[i];
    }
    __syncthreads();
    if (tid < 64) {  // one wave scans the 3072 counts
        int carry = 0;
        for (int base = 0; base < NCELLS; base += 64) {
            int v = cell_start[base + 1 + tid], x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                int y = __shfl_up(x, o, 64);
                if (tid >= o) x += y;
            }
            cell_start[base + 1 + tid] = carry + x;
            carry += __shfl(x, 63, 64);
        }
    }
    __syncthreads();
    for (int i = tid; i < n; i += nthreads) {
        int c = scratch[i];
        if (c >= 0) items[atomicAdd(&cell_start[c], 1)] = i;
    }
    __syncthreads();
    // cell_start[c] now holds the end of cell c: new [c + 1] = old [c], [0] = 0
    for (int c0 = ((NCELLS - 1) / nthreads) * nthreads; c0 >= 0; c0 -= nthreads) {
        const int c = c0 + tid;
        const int v = c < NCELLS ? cell_start[c] : 0;
        __syncthreads();
        if (c < NCELLS) cell_start[c + 1] = v;
        __syncthreads();
    }
    if (tid == 0) cell_start[0] = 0;
    __syncthreads();
    for (int c = tid; c < NCELLS; c += nthreads) {
        int s = cell_start[c], e = cell_start[c + 1];
        for (int a = s + 1; a < e; a++) {
            int v = items[a], b = a - 1;
            while (b >= s && items[b] > v) {
                items[b + 1] = items[b];
                b--;
            }
            items[b + 1] = v;
        }
    }
    __syncthreads();
}

// Frame::GetFeaturesInArea window (Frame.cc:305-327); false if empty.
__device__ __forceinline__ bool grid_window(const FrameConst& fc, float x, float y, float r, int& cx0, int& cx1,
                                            int& cy0, int& cy1) {
    int nMinCellX = max(0, (int)floorf((x - fc.min_x - r) * fc.invW));
    int nMaxCellX = min(GRID_COLS - 1, (int)ceilf((x - fc.min_x + r) * fc.invW));
    int nMinCellY = max(0, (int)floorf((y - fc.min_y - r) * fc.invH));
    int nMaxCellY = min(GRID_ROWS - 1, (int)ceilf((y - fc.min_y + r) * fc.invH));
    if (nMinCellX >= GRID_COLS || nMaxCellX < 0 || nMinCellY >= GRID_ROWS || nMaxCellY < 0) return false;
    cx0 = nMinCellX;
    cx1 = nMaxCellX;
    cy0 = nMinCellY;
    cy1 = nMaxCellY;
    return true;
}
