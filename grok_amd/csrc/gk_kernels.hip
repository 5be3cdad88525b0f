// gk_kernels.hip — MI355X (gfx950) kernels for the JPEG 2000 tile pipeline.
//
// Stage map (reference → kernel), see DESIGN.md:
//   TileProcessor::dcLevelShiftCompress + mct CompressRev   → k_dc_rct_fwd / k_dc_fwd
//   dwt53::encode_and_deinterleave_v/h (WaveletFwd.cpp)      → k_dwt53_fwd_level
//   T1 encode / decode: gk_t1enc.hip, gk_t1dec.hip; 9/7 + ICT: gk_dwt97.hip
//   decompress_tile_53 (WaveletReverse.cpp)                  → k_dwt53_inv_level
//   mct DecompressRev + dcLevelShiftDecompress               → k_rct_inv_dc / k_dc_inv
//
// All kernels are wave64-native: block dims are multiples of 64.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"
#include "gk_xcd.h"
#include "gk_vec.h"

#define LDS_BARRIER() __syncthreads()

// =============================================================================
// Sample access for the caller's planes: int32 (Grok image components) or the
// planar 8/16-bit buffers of grk_compress_tile (TileProcessor.cpp:779-835).
// Four consecutive samples move as one vector access (16 B int32, 4 B u8,
// 8 B u16, gk_vec.h) when the host found every pointer and stride aligned (vec != 0).
// =============================================================================
// DC level shift + RCT (forward).  In: 3 caller planes (stride sin), out: 3
// int32 work planes (stride sout).  mct.cpp:99-146, TileProcessor.cpp:506-535.
// =============================================================================
template <class TI>
__global__ __launch_bounds__(256) void k_dc_rct_fwd(const TI* __restrict__ r_in, const TI* __restrict__ g_in,
                                                    const TI* __restrict__ b_in, uint32_t sin,
                                                    int32_t* __restrict__ y_out, int32_t* __restrict__ u_out,
                                                    int32_t* __restrict__ v_out, uint32_t sout, uint32_t w, uint32_t h,
                                                    int32_t shift, int vec) {
    uint32_t x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    uint32_t y = blockIdx.y;
    if (y >= h || x4 >= w) return;
    const TI* rp = r_in + (size_t)y * sin;
    const TI* gp = g_in + (size_t)y * sin;
    const TI* bp = b_in + (size_t)y * sin;
    int32_t* yp = y_out + (size_t)y * sout;
    int32_t* up = u_out + (size_t)y * sout;
    int32_t* vp = v_out + (size_t)y * sout;
    if (vec && x4 + 3 < w) {
        int4 r = ld4(rp + x4), g = ld4(gp + x4), b = ld4(bp + x4);
        r.x -= shift; r.y -= shift; r.z -= shift; r.w -= shift;
        g.x -= shift; g.y -= shift; g.z -= shift; g.w -= shift;
        b.x -= shift; b.y -= shift; b.z -= shift; b.w -= shift;
        int4 Y, U, V;
        Y.x = (r.x + 2 * g.x + b.x) >> 2; Y.y = (r.y + 2 * g.y + b.y) >> 2;
        Y.z = (r.z + 2 * g.z + b.z) >> 2; Y.w = (r.w + 2 * g.w + b.w) >> 2;
        U.x = b.x - g.x; U.y = b.y - g.y; U.z = b.z - g.z; U.w = b.w - g.w;
        V.x = r.x - g.x; V.y = r.y - g.y; V.z = r.z - g.z; V.w = r.w - g.w;
        st4(yp + x4, Y); st4(up + x4, U); st4(vp + x4, V);
    } else {
        for (uint32_t x = x4; x < w && x < x4 + 4; ++x) {
            int32_t r = (int32_t)rp[x] - shift, g = (int32_t)gp[x] - shift, b = (int32_t)bp[x] - shift;
            yp[x] = (r + 2 * g + b) >> 2; up[x] = b - g; vp[x] = r - g;
        }
    }
}

template <class TI>
__global__ __launch_bounds__(256) void k_dc_fwd(const TI* __restrict__ in, uint32_t sin, int32_t* __restrict__ out,
                                                uint32_t sout, uint32_t w, uint32_t h, int32_t shift) {
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (y >= h || x >= w) return;
    out[(size_t)y * sout + x] = (int32_t)in[(size_t)y * sin + x] - shift;
}

// Inverse RCT + DC shift + clamp (mct.cpp:221-283) into the caller's planes.
template <class TO>
__global__ __launch_bounds__(256) void k_rct_inv_dc(const int32_t* __restrict__ y_in, const int32_t* __restrict__ u_in,
                                                    const int32_t* __restrict__ v_in, uint32_t sin,
                                                    TO* __restrict__ r_out, TO* __restrict__ g_out,
                                                    TO* __restrict__ b_out, uint32_t sout, uint32_t w, uint32_t h,
                                                    int32_t shift, int32_t mn, int32_t mx, int vec) {
    uint32_t x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    uint32_t y = blockIdx.y;
    if (y >= h || x4 >= w) return;
    const int32_t* Yp = y_in + (size_t)y * sin;
    const int32_t* Up = u_in + (size_t)y * sin;
    const int32_t* Vp = v_in + (size_t)y * sin;
    TO* rp = r_out + (size_t)y * sout;
    TO* gp = g_out + (size_t)y * sout;
    TO* bp = b_out + (size_t)y * sout;
    auto cl = [&](int32_t v) { return v < mn ? mn : (v > mx ? mx : v); };
    if (vec && x4 + 3 < w) {
        int4 Y = ld4(Yp + x4), U = ld4(Up + x4), V = ld4(Vp + x4);
        int4 R, G, B;
        G.x = Y.x - ((U.x + V.x) >> 2); G.y = Y.y - ((U.y + V.y) >> 2);
        G.z = Y.z - ((U.z + V.z) >> 2); G.w = Y.w - ((U.w + V.w) >> 2);
        R.x = cl(V.x + G.x + shift); R.y = cl(V.y + G.y + shift); R.z = cl(V.z + G.z + shift); R.w = cl(V.w + G.w + shift);
        B.x = cl(U.x + G.x + shift); B.y = cl(U.y + G.y + shift); B.z = cl(U.z + G.z + shift); B.w = cl(U.w + G.w + shift);
        G.x = cl(G.x + shift); G.y = cl(G.y + shift); G.z = cl(G.z + shift); G.w = cl(G.w + shift);
        st4(rp + x4, R); st4(gp + x4, G); st4(bp + x4, B);
    } else {
        for (uint32_t x = x4; x < w && x < x4 + 4; ++x) {
            int32_t Y = Yp[x], U = Up[x], V = Vp[x];
            int32_t G = Y - ((U + V) >> 2);
            rp[x] = (TO)cl(V + G + shift); gp[x] = (TO)cl(G + shift); bp[x] = (TO)cl(U + G + shift);
        }
    }
}

template <class TO>
__global__ __launch_bounds__(256) void k_dc_inv(const int32_t* __restrict__ in, uint32_t sin, TO* __restrict__ out,
                                                uint32_t sout, uint32_t w, uint32_t h, int32_t shift, int32_t mn,
                                                int32_t mx) {
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (y >= h || x >= w) return;
    int32_t v = in[(size_t)y * sin + x] + shift;
    out[(size_t)y * sout + x] = (TO)(v < mn ? mn : (v > mx ? mx : v));
}

// =============================================================================
// 5/3 reversible DWT, one decomposition level per launch, LDS-tiled.
// Forward (WaveletFwd.cpp:635-960): vertical lifting then horizontal lifting
// on a (TH+3) x (TW+3) LDS tile (2-sample halo before, 1 after, whole-sample
// symmetric extension at the resolution border), outputs written straight into
// the four Mallat quadrants.  Parity 0 (resolution origin even).
// Components run in grid.z (z = component * tiles + tile, GkComps).  Level 1 is
// fused with the sample stage: the forward kernel reads the caller's planes with
// the DC shift and RCT applied on load (k_dwt53_fwd_l1), the inverse kernel writes
// them through the inverse RCT, DC shift and clamp (k_dwt53_inv_l1), so the image
// never makes a separate pass through HBM.
// =============================================================================
#define DWT_TW 128
#ifndef DWT_TH
#define DWT_TH 32
#endif
#define DWT_LW (DWT_TW + 3)
#define DWT_LH (DWT_TH + 3)
typedef int32_t Lds53[DWT_LH][DWT_LW + 1];

__device__ __forceinline__ int mirror(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {   // at most one reflection for halo <= 2 unless n tiny
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

// Visit the forward tile's input positions: rows y0-2 .. y0+TH, cols x0-2 .. x0+TW,
// f(ly, lx, gy, gx) with (gy, gx) mirrored at the resolution border.  4 waves x 64 lanes:
// lane tx walks columns x0 + tx, x0 + 64 + tx of rows ty, ty+4, ... (two 256-byte segments
// aligned to the row's cache lines: starting them at the halo column x0 - 2 made every
// segment touch three 128-byte lines), the halo columns x0-2, x0-1, x0+TW as one extra pass
// (no index division on this path).  Every tile whose TW columns lie inside the resolution
// takes it - rows and halo columns mirrored where they fall outside (a tile-grid border) -
// and only a last, partial tile column the general per-position path.
__device__ __forceinline__ int fwd53_halo_lx(int j) { return j < 2 ? j : DWT_TW + 2; }   // LDS columns 0, 1, TW+2
__device__ __forceinline__ bool fullw53(int x0, int w) { return x0 + DWT_TW <= w; }
template <class F>
__device__ __forceinline__ void fwd53_fill(int x0, int y0, int w, int h, int tid, F f) {
    const int tx = tid & 63, ty = tid >> 6;
    if (fullw53(x0, w)) {
        for (int ly = ty; ly < DWT_LH; ly += 4) {
            const int gy = mirror(y0 - 2 + ly, h);
            f(ly, tx + 2, gy, x0 + tx);
            f(ly, tx + 66, gy, x0 + 64 + tx);
        }
        for (int i = tid; i < 3 * DWT_LH; i += 256) {   // halo columns x0-2, x0-1, x0+TW
            const int ly = i / 3, lx = fwd53_halo_lx(i % 3);
            f(ly, lx, mirror(y0 - 2 + ly, h), mirror(x0 - 2 + lx, w));
        }
    } else {
        for (int i = tid; i < DWT_LH * DWT_LW; i += 256) {
            const int ly = i / DWT_LW, lx = i % DWT_LW;
            f(ly, lx, mirror(y0 - 2 + ly, h), mirror(x0 - 2 + lx, w));
        }
    }
}

// Forward lifting of one loaded tile (barriers inside: every thread of the block calls it).
__device__ __forceinline__ void fwd53_lift(Lds53& T, int w, int h, int tid) {
    const int tx = tid & 63, ty = tid >> 6;
    if (h > 1) {
        // vertical predict: odd absolute rows y in [y0-1, y0+TH-1]  (local ly = y - y0 + 2, odd y <=> ly odd)
        // (columns 0..127 by every lane, the halo columns 128..130 as one extra pass: a loop
        // tail that only a few lanes enter would cost a full pass per row)
        for (int k = ty; k <= DWT_TH / 2; k += 4) {
            const int ly = 1 + 2 * k;   // y = y0 - 1 + 2k
            for (int lx = tx; lx < 128; lx += 64) T[ly][lx] -= (T[ly - 1][lx] + T[ly + 1][lx]) >> 1;
        }
        if (tid < 3 * (DWT_TH / 2 + 1)) {
            const int ly = 1 + 2 * (tid / 3), lx = 128 + tid % 3;
            T[ly][lx] -= (T[ly - 1][lx] + T[ly + 1][lx]) >> 1;
        }
        LDS_BARRIER();
        // vertical update: even rows y in [y0, y0+TH-2]: ly = 2 + 2k
        for (int k = ty; k < DWT_TH / 2; k += 4) {
            const int ly = 2 + 2 * k;
            for (int lx = tx; lx < 128; lx += 64) T[ly][lx] += (T[ly - 1][lx] + T[ly + 1][lx] + 2) >> 2;
        }
        if (tid < 3 * (DWT_TH / 2)) {
            const int ly = 2 + 2 * (tid / 3), lx = 128 + tid % 3;
            T[ly][lx] += (T[ly - 1][lx] + T[ly + 1][lx] + 2) >> 2;
        }
        LDS_BARRIER();
    }
    if (w > 1) {
        // horizontal predict on rows ly in [2, TH+2): odd cols lx = 1 + 2k, k in [0, TW/2]
        for (int ly = 2 + ty; ly < DWT_TH + 2; ly += 4) {
            const int lx = 1 + 2 * tx;
            T[ly][lx] -= (T[ly][lx - 1] + T[ly][lx + 1]) >> 1;
        }
        if (tid < DWT_TH) {   // k = TW/2 (lx = TW + 1) of every row
            const int ly = 2 + tid, lx = DWT_TW + 1;
            T[ly][lx] -= (T[ly][lx - 1] + T[ly][lx + 1]) >> 1;
        }
        LDS_BARRIER();
        for (int ly = 2 + ty; ly < DWT_TH + 2; ly += 4) {
            const int lx = 2 + 2 * tx;   // k = tx in [0, TW/2)
            T[ly][lx] += (T[ly][lx - 1] + T[ly][lx + 1] + 2) >> 2;
        }
        LDS_BARRIER();
    }
}

// scatter to quadrants: lane tx writes L and H sample k = tx of each row (coalesced rows)
__device__ __forceinline__ void fwd53_store(const Lds53& T, int32_t* __restrict__ dst, uint32_t dstride, int x0, int y0,
                                            int w, int h, int tid) {
    const int tx = tid & 63, ty = tid >> 6;
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    const bool full = x0 + DWT_TW <= w && y0 + DWT_TH <= h;
    for (int ry = ty; ry < DWT_TH; ry += 4) {
        const int gy = y0 + ry;
        if (!full && gy >= h) break;
        const int oy = ((gy & 1) == 0) ? (gy >> 1) : (snh + (gy >> 1));
        int32_t* drow = dst + (size_t)oy * dstride;
        const int gxl = x0 + 2 * tx;
        if (full || gxl < w) drow[gxl >> 1] = T[ry + 2][2 + 2 * tx];
        if (full || gxl + 1 < w) drow[snw + (gxl >> 1)] = T[ry + 2][3 + 2 * tx];
    }
}

// One level, cpw components per workgroup (grid z: tile + count * component group).  With
// several, full-width tiles load the next component's input into registers (the positions
// fwd53_fill's full-width path visits) while the current one lifts, as k_dwt53_inv_l1 does;
// the launcher takes one component per workgroup when the grid would not fill the chip.
__global__ __launch_bounds__(256) void k_dwt53_fwd_level(const int32_t* __restrict__ src, uint32_t sstride,
                                                         int32_t* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h, GkTiles tb, GkComps cs, uint32_t cpw) {
    __shared__ Lds53 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z % tb.count(), c0 = bi.z / tb.count() * cpw, c1 = min(cs.n, c0 + cpw);
    src += tb.offset(tile, sstride);
    dst += tb.offset(tile, dstride);
    const int x0 = bi.x * DWT_TW, y0 = bi.y * DWT_TH, tid = threadIdx.x;
    const int tx = tid & 63, ty = tid >> 6;
    constexpr int PF_ROWS = (DWT_LH + 3) / 4;
    int32_t PF[2 * PF_ROWS + 1];
    const bool inner = fullw53(x0, (int)w);
    auto fetch = [&](const int32_t* sc) {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < DWT_LH) {
                const int32_t* r = sc + (size_t)mirror(y0 - 2 + ly, (int)h) * sstride + x0 + tx;
                PF[2 * m] = r[0];
                PF[2 * m + 1] = r[64];
            }
        }
        if (tid < 3 * DWT_LH) {   // halo columns x0-2, x0-1, x0+TW (as fwd53_fill)
            const int ly = tid / 3, lx = fwd53_halo_lx(tid % 3);
            PF[2 * PF_ROWS] = sc[(size_t)mirror(y0 - 2 + ly, (int)h) * sstride + mirror(x0 - 2 + lx, (int)w)];
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < DWT_LH) { T[ly][tx + 2] = PF[2 * m]; T[ly][tx + 66] = PF[2 * m + 1]; }
        }
        if (tid < 3 * DWT_LH) T[tid / 3][fwd53_halo_lx(tid % 3)] = PF[2 * PF_ROWS];
    };
    if (inner) fetch(src + c0 * cs.cstride);
    for (uint32_t c = c0; c < c1; ++c) {
        if (c != c0) LDS_BARRIER();   // the previous component's stores have read the tile
        const int32_t* sc = src + c * cs.cstride;
        if (inner) put();
        else fwd53_fill(x0, y0, (int)w, (int)h, tid,
                        [&](int ly, int lx, int gy, int gx) { T[ly][lx] = sc[(size_t)gy * sstride + gx]; });
        LDS_BARRIER();
        if (inner && c + 1 < c1) fetch(sc + cs.cstride);
        fwd53_lift(T, (int)w, (int)h, tid);
        fwd53_store(T, dst + c * cs.cstride, dstride, x0, y0, (int)w, (int)h, tid);
    }
}

// Level 1 from the caller's planes: DC shift (TileProcessor.cpp:506-535) and, for NC = 3,
// the RCT (mct.cpp:99-146) on load; outputs into the level-1 planes of the NC components
// (dst + c * cstride).  One LDS tile: Y is transformed first while each thread keeps the U
// and V of its input positions in registers, then U, then V go through the same tile, so a
// workgroup needs one LDS tile instead of three (occupancy).  Interior tiles read the planes
// four samples per lane: five groups of four consecutive samples per thread cover the 35 x 128
// main positions (one vector load per group and plane, 128 contiguous samples per half wave),
// one more slot the 3 x 35 halo columns; edge tiles take L1_EDGE mirrored positions per thread.
#define L1_GROUPS 5                                 // ceil(35 x 32 / 256) groups of four
#define L1_SLOTS (4 * L1_GROUPS + 1)                // + one halo column slot
#define L1_EDGE ((DWT_LH * DWT_LW + 255) / 256)     // positions per thread on edge tiles
static_assert(L1_EDGE <= L1_SLOTS, "edge-tile positions fit the register slots");
static_assert(32 * DWT_LH <= 256 * L1_GROUPS, "interior groups fit");
template <class F>   // f(group, ly, lx): interior groups of four positions (ly, lx .. lx + 3)
__device__ __forceinline__ void fwd53_groups(int tid, F f) {
#pragma unroll
    for (int g = 0; g < L1_GROUPS; ++g) {
        const int i = tid + 256 * g;
        if (i < 32 * DWT_LH) f(g, i >> 5, 2 + 4 * (i & 31));
    }
}

template <class TI, int NC>
__global__ __launch_bounds__(256) void k_dwt53_fwd_l1(GkPtr3 in, uint32_t sin, int32_t* __restrict__ dst,
                                                      uint64_t cstride, uint32_t dstride, uint32_t w, uint32_t h,
                                                      GkTiles tb, int32_t shift, int vec) {
    __shared__ Lds53 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z;
    const uint64_t io = tb.offset(tile, sin);
    const TI* p0 = (const TI*)in.p[0] + io;
    const TI* p1 = (const TI*)in.p[NC == 3 ? 1 : 0] + io;
    const TI* p2 = (const TI*)in.p[NC == 3 ? 2 : 0] + io;
    dst += tb.offset(tile, dstride);
    const int x0 = bi.x * DWT_TW, y0 = bi.y * DWT_TH, tid = threadIdx.x;
    int32_t U[L1_SLOTS], V[L1_SLOTS];
    auto put = [&](int k, int ly, int lx, int32_t r0, int32_t g0, int32_t b0) {
        if (NC == 3) {
            const int32_t r = r0 - shift, g = g0 - shift, b = b0 - shift;
            T[ly][lx] = (r + 2 * g + b) >> 2;
            U[k] = b - g;
            V[k] = r - g;
        } else {
            T[ly][lx] = r0 - shift;
        }
    };
    const bool inner = fullw53(x0, (int)w);   // (rows and halo columns mirrored)
    if (inner) {
        // (x0 is a multiple of 128, so every group is aligned when the plane rows are)
        const bool v = vec && al4(p0) && al4(p1) && al4(p2);
        fwd53_groups(tid, [&](int g, int ly, int lx) {
            const size_t i = (size_t)mirror(y0 - 2 + ly, (int)h) * sin + (x0 - 2 + lx);
            const int4 a = ld4v(p0 + i, v);
            const int4 b = NC == 3 ? ld4v(p1 + i, v) : a, c = NC == 3 ? ld4v(p2 + i, v) : a;
            put(4 * g, ly, lx, a.x, b.x, c.x);
            put(4 * g + 1, ly, lx + 1, a.y, b.y, c.y);
            put(4 * g + 2, ly, lx + 2, a.z, b.z, c.z);
            put(4 * g + 3, ly, lx + 3, a.w, b.w, c.w);
        });
        if (tid < 3 * DWT_LH) {   // halo columns x0-2, x0-1, x0+TW
            const int ly = tid / 3, lx = fwd53_halo_lx(tid % 3);
            const size_t i = (size_t)mirror(y0 - 2 + ly, (int)h) * sin + mirror(x0 - 2 + lx, (int)w);
            put(4 * L1_GROUPS, ly, lx, (int32_t)p0[i], (int32_t)p1[i], (int32_t)p2[i]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < L1_EDGE; ++k) {
            const int i = tid + 256 * k;
            if (i < DWT_LH * DWT_LW) {
                const int ly = i / DWT_LW, lx = i % DWT_LW;
                const size_t o = (size_t)mirror(y0 - 2 + ly, (int)h) * sin + mirror(x0 - 2 + lx, (int)w);
                put(k, ly, lx, (int32_t)p0[o], (int32_t)p1[o], (int32_t)p2[o]);
            }
        }
    }
    LDS_BARRIER();
    fwd53_lift(T, (int)w, (int)h, tid);
    fwd53_store(T, dst, dstride, x0, y0, (int)w, (int)h, tid);
    if (NC == 3) {
#pragma unroll
        for (int c = 1; c < 3; ++c) {
            LDS_BARRIER();   // the previous component's stores have read the tile
            if (inner) {
                fwd53_groups(tid, [&](int g, int ly, int lx) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) T[ly][lx + j] = c == 1 ? U[4 * g + j] : V[4 * g + j];
                });
                if (tid < 3 * DWT_LH) T[tid / 3][fwd53_halo_lx(tid % 3)] = c == 1 ? U[4 * L1_GROUPS] : V[4 * L1_GROUPS];
            } else {
#pragma unroll
                for (int k = 0; k < L1_EDGE; ++k) {
                    const int i = tid + 256 * k;
                    if (i < DWT_LH * DWT_LW) T[i / DWT_LW][i % DWT_LW] = c == 1 ? U[k] : V[k];
                }
            }
            LDS_BARRIER();
            fwd53_lift(T, (int)w, (int)h, tid);
            fwd53_store(T, dst + c * cstride, dstride, x0, y0, (int)w, (int)h, tid);
        }
    }
}

// Inverse 5/3 level (WaveletReverse.cpp:802-879): horizontal then vertical,
// on the interleaved signal with symmetric extension.  Output tile rows
// y0..y0+TH-1; needs interleaved rows y0-1..y0+TH+1 and cols x0-1..x0+TW+1.
#define IDWT_LW (DWT_TW + 3)
#define IDWT_LH (DWT_TH + 3)

// Visit the inverse tile's input: interleaved position (ly, lx) = (y0-1+ly, x0-1+lx) comes
// from Mallat position (sy, sx): f(ly, lx, sy, sx).
template <class F>
__device__ __forceinline__ void inv53_fill(int x0, int y0, int w, int h, int tid, F f) {
    const int tx = tid & 63, ty = tid >> 6;
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    auto sxo = [&](int gx) { return (gx & 1) ? (snw + (gx >> 1)) : (gx >> 1); };
    if (fullw53(x0, w)) {   // (rows and halo columns mirrored, as fwd53_fill)
        // interleaved column gx = x0 - 1 + lx: odd lx <=> even gx (L sample x0/2 + k, lx = 1 + 2k),
        // even lx <=> odd gx (H sample x0/2 - 1 + k, lx = 2k).  The main pass reads L samples
        // x0/2 + tx and H samples x0/2 + tx (lx = 2 + 2 tx), both segments starting on a line
        // boundary when the band starts on one (snw a multiple of 32)
        for (int ly = ty; ly < IDWT_LH; ly += 4) {
            const int gy = mirror(y0 - 1 + ly, h);
            const int sy = (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1);
            f(ly, 1 + 2 * tx, sy, (x0 >> 1) + tx);
            f(ly, 2 + 2 * tx, sy, snw + (x0 >> 1) + tx);
        }
        for (int i = tid; i < 3 * IDWT_LH; i += 256) {   // lx 0 (gx x0 - 1), 129 (x0 + TW), 130 (x0 + TW + 1)
            const int ly = i / 3, j = i % 3, gy = mirror(y0 - 1 + ly, h);
            const int sy = (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1);
            const int lx = j ? 128 + j : 0;
            f(ly, lx, sy, sxo(mirror(x0 - 1 + lx, w)));
        }
    } else {
        for (int i = tid; i < IDWT_LH * IDWT_LW; i += 256) {
            const int ly = i / IDWT_LW, lx = i % IDWT_LW;
            const int gy = mirror(y0 - 1 + ly, h), gx = mirror(x0 - 1 + lx, w);
            f(ly, lx, (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1), sxo(gx));
        }
    }
}

// k_dwt53_inv_l1's tile: rows start 3 dwords in, so output column c (LDS column c + 1) of a
// 4-column group sits on a 16-byte boundary and a group is one ds_read_b128
struct alignas(16) Lds53A {
    int32_t a[DWT_LH][DWT_LW + 5];
    __device__ __forceinline__ int32_t* operator[](int r) { return a[r] + 3; }
    __device__ __forceinline__ const int32_t* operator[](int r) const { return a[r] + 3; }
};
template <class TT>
__device__ __forceinline__ void inv53_lift(TT& T, int w, int h, int tid) {
    const int tx = tid & 63, ty = tid >> 6;
    if (w > 1) {
        // horizontal step 1: even interleaved cols x (lx = x - x0 + 1): x even <=> lx odd, lx in [1, TW+1]
        for (int ly = ty; ly < IDWT_LH; ly += 4) {
            const int lx = 1 + 2 * tx;
            T[ly][lx] -= (T[ly][lx - 1] + T[ly][lx + 1] + 2) >> 2;
        }
        if (tid < IDWT_LH) {   // k = TW/2 (lx = TW + 1) of every row
            const int ly = tid, lx = DWT_TW + 1;
            T[ly][lx] -= (T[ly][lx - 1] + T[ly][lx + 1] + 2) >> 2;
        }
        LDS_BARRIER();
        // step 2: odd cols x in [x0+1, x0+TW-1]: lx = 2 + 2k, k = tx
        for (int ly = ty; ly < IDWT_LH; ly += 4) {
            const int lx = 2 + 2 * tx;
            T[ly][lx] += (T[ly][lx - 1] + T[ly][lx + 1]) >> 1;
        }
        LDS_BARRIER();
    }
    if (h > 1) {
        for (int k = ty; k <= DWT_TH / 2; k += 4) {
            const int ly = 1 + 2 * k;
            for (int lx = 1 + tx; lx <= DWT_TW; lx += 64) T[ly][lx] -= (T[ly - 1][lx] + T[ly + 1][lx] + 2) >> 2;
        }
        LDS_BARRIER();
        for (int k = ty; k < DWT_TH / 2; k += 4) {
            const int ly = 2 + 2 * k;
            for (int lx = 1 + tx; lx <= DWT_TW; lx += 64) T[ly][lx] += (T[ly - 1][lx] + T[ly + 1][lx]) >> 1;
        }
        LDS_BARRIER();
    }
}

// One level, cpw components per workgroup with the next one's input prefetched (as
// k_dwt53_fwd_level)
__global__ __launch_bounds__(256) void k_dwt53_inv_level(const int32_t* __restrict__ src, uint32_t sstride,
                                                         int32_t* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h, GkTiles tb, GkComps cs, uint32_t cpw) {
    __shared__ Lds53 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z % tb.count(), c0 = bi.z / tb.count() * cpw, c1 = min(cs.n, c0 + cpw);
    src += tb.offset(tile, sstride);
    dst += tb.offset(tile, dstride);
    const int x0 = bi.x * DWT_TW, y0 = bi.y * DWT_TH, tid = threadIdx.x;
    const int tx = tid & 63, ty = tid >> 6;
    constexpr int PF_ROWS = (IDWT_LH + 3) / 4;
    int32_t PF[2 * PF_ROWS + 1];
    const bool inner = fullw53(x0, (int)w);
    const int snw = ((int)w + 1) >> 1, snh = ((int)h + 1) >> 1;
    auto srow = [&](int ly) {
        const int gy = mirror(y0 - 1 + ly, (int)h);
        return (size_t)((gy & 1) ? (snh + (gy >> 1)) : (gy >> 1)) * sstride;
    };
    auto fetch = [&](const int32_t* sc) {   // (inv53_fill's full-width positions)
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < IDWT_LH) {
                const int32_t* r = sc + srow(ly) + (x0 >> 1) + tx;
                PF[2 * m] = r[0];
                PF[2 * m + 1] = r[snw];
            }
        }
        if (tid < 3 * IDWT_LH) {
            const int ly = tid / 3, j = tid % 3, lx = j ? 128 + j : 0;
            const int gx = mirror(x0 - 1 + lx, (int)w);
            PF[2 * PF_ROWS] = sc[srow(ly) + ((gx & 1) ? (snw + (gx >> 1)) : (gx >> 1))];
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < IDWT_LH) { T[ly][1 + 2 * tx] = PF[2 * m]; T[ly][2 + 2 * tx] = PF[2 * m + 1]; }
        }
        if (tid < 3 * IDWT_LH) { const int j = tid % 3; T[tid / 3][j ? 128 + j : 0] = PF[2 * PF_ROWS]; }
    };
    const bool full = x0 + DWT_TW <= (int)w && y0 + DWT_TH <= (int)h;
    if (inner) fetch(src + c0 * cs.cstride);
    for (uint32_t c = c0; c < c1; ++c) {
        if (c != c0) LDS_BARRIER();   // the previous component's stores have read the tile
        const int32_t* sc = src + c * cs.cstride;
        if (inner) put();
        else inv53_fill(x0, y0, (int)w, (int)h, tid,
                        [&](int ly, int lx, int sy, int sx) { T[ly][lx] = sc[(size_t)sy * sstride + sx]; });
        LDS_BARRIER();
        if (inner && c + 1 < c1) fetch(sc + cs.cstride);
        inv53_lift(T, (int)w, (int)h, tid);
        int32_t* dc = dst + c * cs.cstride;
        for (int ry = ty; ry < DWT_TH; ry += 4) {
            const int gy = y0 + ry;
            if (!full && gy >= (int)h) break;
            int32_t* drow = dc + (size_t)gy * dstride + x0;
            for (int cc = tx; cc < DWT_TW; cc += 64)
                if (full || x0 + cc < (int)w) drow[cc] = T[ry + 1][cc + 1];
        }
    }
}

// Last inverse level into the caller's planes: inverse RCT for NC = 3 (mct.cpp:221-283),
// DC shift and clamp (TileProcessor.cpp:457-504), samples of type TO, only inside the
// output window (region coordinates [wx0, wx1) x [wy0, wy1); out.p[c] addresses (wx0, wy0)).
// One LDS tile: the Y and U results of each thread's 16 output samples wait in registers
// while the next component goes through the tile.  A thread owns four groups of four
// consecutive columns (row i >> 5, columns 4 (i & 31) .. + 3 of group i = tid + 256 j), written
// as one vector store per plane where the window and the planes allow.
template <class TO, int NC>
__global__ __launch_bounds__(256) void k_dwt53_inv_l1(const int32_t* __restrict__ src, uint64_t cstride, uint32_t sstride,
                                                      GkPtr3 out, uint32_t ostride, GkWin win, uint32_t w, uint32_t h,
                                                      GkTiles tb, int32_t shift, int32_t mn, int32_t mx, int vec) {
    __shared__ Lds53A T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z;
    src += tb.offset(tile, sstride);
    int32_t ox, oy;
    tb.origin(tile, ox, oy);
    const int x0 = bi.x * DWT_TW, y0 = bi.y * DWT_TH, tid = threadIdx.x;
    static_assert(DWT_TW * DWT_TH == 4 * 4 * 256, "four groups of four per thread");
    int32_t R0[16], R1[16];
    // Full-width tiles: the next component's input is loaded into registers (PF, the positions
    // inv53_fill's full-width path visits) while the current one lifts, so its HBM latency
    // overlaps the lifting instead of following it.
    constexpr int PF_ROWS = (IDWT_LH + 3) / 4;
    int32_t PF[2 * PF_ROWS + 1];
    const bool inner = fullw53(x0, (int)w);
    const int tx = tid & 63, ty = tid >> 6;
    const int snw = ((int)w + 1) >> 1, snh = ((int)h + 1) >> 1;
    auto srow = [&](int ly) {
        const int gy = mirror(y0 - 1 + ly, (int)h);
        return (size_t)((gy & 1) ? (snh + (gy >> 1)) : (gy >> 1)) * sstride;
    };
    auto fetch = [&](const int32_t* sc) {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < IDWT_LH) {
                const int32_t* r = sc + srow(ly) + (x0 >> 1) + tx;
                PF[2 * m] = r[0];
                PF[2 * m + 1] = r[snw];
            }
        }
        if (tid < 3 * IDWT_LH) {   // lx 0, 129, 130 (as inv53_fill)
            const int ly = tid / 3, j = tid % 3, lx = j ? 128 + j : 0;
            const int gx = mirror(x0 - 1 + lx, (int)w);
            PF[2 * PF_ROWS] = sc[srow(ly) + ((gx & 1) ? (snw + (gx >> 1)) : (gx >> 1))];
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < IDWT_LH) { T[ly][1 + 2 * tx] = PF[2 * m]; T[ly][2 + 2 * tx] = PF[2 * m + 1]; }
        }
        if (tid < 3 * IDWT_LH) { const int j = tid % 3; T[tid / 3][j ? 128 + j : 0] = PF[2 * PF_ROWS]; }
    };
    if (inner) fetch(src);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (c) LDS_BARRIER();   // the previous component's samples have been read
        const int32_t* sc = src + c * cstride;
        if (inner) put();
        else inv53_fill(x0, y0, (int)w, (int)h, tid,
                        [&](int ly, int lx, int sy, int sx) { T[ly][lx] = sc[(size_t)sy * sstride + sx]; });
        LDS_BARRIER();
        if (inner && c + 1 < NC) fetch(sc + cstride);
        inv53_lift(T, (int)w, (int)h, tid);
        if (c + 1 < NC) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = tid + 256 * j;
                const int4 v = *(const int4*)&T[(i >> 5) + 1][4 * (i & 31) + 1];
                int32_t* R = c == 0 ? R0 : R1;
                R[4 * j] = v.x; R[4 * j + 1] = v.y; R[4 * j + 2] = v.z; R[4 * j + 3] = v.w;
            }
        }
    }
    TO* o0 = (TO*)out.p[0];
    TO* o1 = (TO*)out.p[NC == 3 ? 1 : 0];
    TO* o2 = (TO*)out.p[NC == 3 ? 2 : 0];
    auto cl = [&](int32_t v) { return v < mn ? mn : (v > mx ? mx : v); };
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = tid + 256 * j, ry = i >> 5, rx = 4 * (i & 31);
        const int gy = y0 + ry, Y = oy + gy, gx = x0 + rx, X = ox + gx;
        if (gy >= (int)h || Y < win.y0 || Y >= win.y1) continue;
        int32_t r[4], g[4], b[4];
        const int4 lv = *(const int4*)&T[ry + 1][rx + 1];
        const int32_t lastv[4] = {lv.x, lv.y, lv.z, lv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int32_t last = lastv[e];
            if (NC == 3) {
                const int32_t G = R0[4 * j + e] - ((R1[4 * j + e] + last) >> 2);
                r[e] = cl(last + G + shift);
                g[e] = cl(G + shift);
                b[e] = cl(R1[4 * j + e] + G + shift);
            } else {
                r[e] = cl(last + shift);
            }
        }
        const size_t o = (size_t)(Y - win.y0) * ostride + (X - win.x0);
        if (vec && gx + 3 < (int)w && X >= win.x0 && X + 3 < win.x1 && ((X - win.x0) & 3) == 0) {
            st4(o0 + o, make_int4(r[0], r[1], r[2], r[3]));
            if (NC == 3) { st4(o1 + o, make_int4(g[0], g[1], g[2], g[3])); st4(o2 + o, make_int4(b[0], b[1], b[2], b[3])); }
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (gx + e >= (int)w || X + e < win.x0 || X + e >= win.x1) continue;
                o0[o + e] = (TO)r[e];
                if (NC == 3) { o1[o + e] = (TO)g[e]; o2[o + e] = (TO)b[e]; }
            }
        }
    }
}

// =============================================================================
// Byte gather for codestream assembly and decode staging.
// seg: (src_off, dst_off, len) triples; one wave per segment.
// =============================================================================
// Bytes up to the next 16-byte boundary of the destination go one per lane; then every lane
// stores 16 aligned bytes per iteration, built from the covering source dwords with alignbyte
// (a source offset need not share the destination's alignment); the tail goes one per lane.
__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                const uint64_t* __restrict__ seg, uint32_t nseg) {
    uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= nseg) return;
    const uint64_t so = seg[3 * s], d = seg[3 * s + 1];
    uint64_t n = seg[3 * s + 2];
    const int lane = threadIdx.x & 63;
    const uint8_t* sp = src + so;
    uint8_t* dp = dst + d;
    const uint64_t head = min(n, (uint64_t)((16 - (d & 15)) & 15));
    if ((uint64_t)lane < head) dp[lane] = sp[lane];
    sp += head; dp += head; n -= head;
    const uint64_t nch = n / 16;
    const uint32_t sh = (uint32_t)((uintptr_t)sp & 3);
    const uint32_t* sw = (const uint32_t*)((uintptr_t)sp & ~(uintptr_t)3);
    for (uint64_t c = lane; c < nch; c += 64) {
        const uint32_t* w = sw + 4 * c;
        const uint32_t a0 = w[0], a1 = w[1], a2 = w[2], a3 = w[3], a4 = sh ? w[4] : 0u;
        uint4 v;
        v.x = __builtin_amdgcn_alignbyte(a1, a0, sh);
        v.y = __builtin_amdgcn_alignbyte(a2, a1, sh);
        v.z = __builtin_amdgcn_alignbyte(a3, a2, sh);
        v.w = __builtin_amdgcn_alignbyte(a4, a3, sh);
        *(uint4*)(dp + 16 * c) = v;
    }
    for (uint64_t i = nch * 16 + lane; i < n; i += 64) dp[i] = sp[i];
}

// =============================================================================
// Host launch wrappers (declared in gk_launch.h).  All launches are async on
// the given stream; none allocates or synchronises (graph-capturable).
// =============================================================================
#include "gk_launch.h"

// vector path: every plane pointer aligned to 4 samples of its type, strides multiples of 4
static int vec_ok(uint32_t es_a, const void* a0, const void* a1, const void* a2, uint32_t sa, uint32_t es_b,
                  const void* b0, const void* b1, const void* b2, uint32_t sb) {
    auto al = [](const void* p, uint32_t es) { return ((uintptr_t)p % (4 * es)) == 0; };
    return al(a0, es_a) && al(a1, es_a) && al(a2, es_a) && al(b0, es_b) && al(b1, es_b) && al(b2, es_b) &&
           (sa & 3) == 0 && (sb & 3) == 0;
}
void gk_launch_dc_rct_fwd(hipStream_t st, int stype, const void* r, const void* g, const void* b, uint32_t sin,
                          int32_t* y, int32_t* u, int32_t* v, uint32_t sout, uint32_t w, uint32_t h, int32_t shift) {
    if (!w || !h) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + 1023) / 1024, h);
    const int vec = vec_ok(gk_sample_size(stype), r, g, b, sin, 4, y, u, v, sout);
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_rct_fwd<T>, grid, dim3(256), 0, st, (const T*)r, (const T*)g, (const T*)b, sin, y, u, v,
                           sout, w, h, shift, vec))
}
void gk_launch_dc_fwd(hipStream_t st, int stype, const void* in, uint32_t sin, int32_t* out, uint32_t sout, uint32_t w,
                      uint32_t h, int32_t shift) {
    if (!w || !h) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + 255) / 256, h);
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_fwd<T>, grid, dim3(256), 0, st, (const T*)in, sin, out, sout, w, h, shift))
}
void gk_launch_rct_inv_dc(hipStream_t st, const int32_t* y, const int32_t* u, const int32_t* v, uint32_t sin, int stype,
                          void* r, void* g, void* b, uint32_t sout, uint32_t w, uint32_t h, int32_t shift,
                          int32_t mn, int32_t mx) {
    if (!w || !h) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + 1023) / 1024, h);
    const int vec = vec_ok(4, y, u, v, sin, gk_sample_size(stype), r, g, b, sout);
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_rct_inv_dc<T>, grid, dim3(256), 0, st, y, u, v, sin, (T*)r, (T*)g, (T*)b, sout, w, h, shift,
                           mn, mx, vec))
}
void gk_launch_dc_inv(hipStream_t st, const int32_t* in, uint32_t sin, int stype, void* out, uint32_t sout, uint32_t w,
                      uint32_t h, int32_t shift, int32_t mn, int32_t mx) {
    if (!w || !h) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + 255) / 256, h);
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_inv<T>, grid, dim3(256), 0, st, in, sin, (T*)out, sout, w, h, shift, mn, mx))
}
static uint32_t comps_in_grid(GkTiles tb, GkComps cs) { return tb.count() * cs.n <= 65535u ? cs.n : 1u; }
// components per workgroup of a level launch.  One, unless `multi` (the kernel measured faster
// with the next component prefetched) and the grid still gives every CU 8 workgroups of all the
// components: C2 (5/3) levels 2-5 one per workgroup 125 / 139 µs forward / inverse per step,
// all three 146 / 163 (the register-staged fill alone is the gain over the per-position fill,
// 164 / 193); C3 (9/7) forward 210 / 222 µs with all / one.  GK_DWT_CPW=1 / 3 forces one / all.
uint32_t gk_dwt_cpw(uint32_t wgs, uint32_t n, bool multi) {
    static const int force = getenv("GK_DWT_CPW") ? atoi(getenv("GK_DWT_CPW")) : 0;
    if (force == 1) multi = false;
    if (force > 1) multi = true;
    return (multi && n > 1 && wgs >= 8u * 256u) ? n : 1u;
}
void gk_launch_dwt53_fwd(hipStream_t st, const int32_t* src, uint32_t sstride, int32_t* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb, GkComps cs) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    const uint32_t gx = (w + DWT_TW - 1) / DWT_TW, gy = (h + DWT_TH - 1) / DWT_TH;
    const uint32_t cpw = gk_dwt_cpw(gx * gy * tb.count(), cs.n, false);
    const uint32_t ng = cpw > 1 ? cs.n : comps_in_grid(tb, cs);   // components per launch
    for (uint32_t c = 0; c < cs.n; c += ng) {
        GkComps g = cs; g.n = ng;
        dim3 grid(gx, gy, tb.count() * (ng / cpw));
        hipLaunchKernelGGL(k_dwt53_fwd_level, grid, dim3(256), 0, st, src + c * cs.cstride, sstride, dst + c * cs.cstride,
                           dstride, w, h, tb, g, cpw);
    }
}
void gk_launch_dwt53_inv(hipStream_t st, const int32_t* src, uint32_t sstride, int32_t* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb, GkComps cs) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    const uint32_t gx = (w + DWT_TW - 1) / DWT_TW, gy = (h + DWT_TH - 1) / DWT_TH;
    const uint32_t cpw = gk_dwt_cpw(gx * gy * tb.count(), cs.n, false);
    const uint32_t ng = cpw > 1 ? cs.n : comps_in_grid(tb, cs);
    for (uint32_t c = 0; c < cs.n; c += ng) {
        GkComps g = cs; g.n = ng;
        dim3 grid(gx, gy, tb.count() * (ng / cpw));
        hipLaunchKernelGGL(k_dwt53_inv_level, grid, dim3(256), 0, st, src + c * cs.cstride, sstride, dst + c * cs.cstride,
                           dstride, w, h, tb, g, cpw);
    }
}
void gk_launch_dwt53_fwd_l1(hipStream_t st, int stype, int nc, GkPtr3 in, uint32_t sin, int32_t* dst, uint64_t cstride,
                            uint32_t dstride, uint32_t w, uint32_t h, GkTiles tb, int32_t shift) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + DWT_TW - 1) / DWT_TW, (h + DWT_TH - 1) / DWT_TH, tb.count());
    const int vec = (sin & 3) == 0;   // (the kernel checks each tile's row pointers)
    if (nc == 3)
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt53_fwd_l1<T, 3>), grid, dim3(256), 0, st, in, sin, dst,
                                                        cstride, dstride, w, h, tb, shift, vec))
    else
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt53_fwd_l1<T, 1>), grid, dim3(256), 0, st, in, sin, dst,
                                                        cstride, dstride, w, h, tb, shift, vec))
}
void gk_launch_dwt53_inv_l1(hipStream_t st, int stype, int nc, const int32_t* src, uint64_t cstride, uint32_t sstride,
                            GkPtr3 out, uint32_t ostride, GkWin win, uint32_t w, uint32_t h, GkTiles tb, int32_t shift,
                            int32_t mn, int32_t mx) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + DWT_TW - 1) / DWT_TW, (h + DWT_TH - 1) / DWT_TH, tb.count());
    const int vec = gk_vec_ok(gk_sample_size(stype), out, nc, ostride);
    if (nc == 3)
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt53_inv_l1<T, 3>), grid, dim3(256), 0, st, src, cstride,
                                                        sstride, out, ostride, win, w, h, tb, shift, mn, mx, vec))
    else
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt53_inv_l1<T, 1>), grid, dim3(256), 0, st, src, cstride,
                                                        sstride, out, ostride, win, w, h, tb, shift, mn, mx, vec))
}
void gk_launch_gather(hipStream_t st, const uint8_t* src, uint8_t* dst, const uint64_t* seg, uint32_t nseg) {
    if (!nseg) return;
    hipLaunchKernelGGL(k_gather, dim3((nseg + 3) / 4), dim3(256), 0, st, src, dst, seg, nseg);
}
