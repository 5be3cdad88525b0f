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

#define LDS_BARRIER() __syncthreads()

// =============================================================================
// Sample access for the caller's planes: int32 (Grok image components) or the
// planar 8/16-bit buffers of grk_compress_tile (TileProcessor.cpp:779-835).
// Four consecutive samples move as one vector access (16 B int32, 4 B u8,
// 8 B u16) when the host found every pointer and stride aligned (vec != 0).
// =============================================================================
__device__ __forceinline__ int4 ld4(const int32_t* p) { return *(const int4*)p; }
__device__ __forceinline__ int4 ld4(const uint8_t* p) { const uchar4 v = *(const uchar4*)p; return make_int4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ int4 ld4(const int8_t* p) { const char4 v = *(const char4*)p; return make_int4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ int4 ld4(const uint16_t* p) { const ushort4 v = *(const ushort4*)p; return make_int4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ int4 ld4(const int16_t* p) { const short4 v = *(const short4*)p; return make_int4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ void st4(int32_t* p, int4 v) { *(int4*)p = v; }
__device__ __forceinline__ void st4(uint8_t* p, int4 v) { *(uchar4*)p = make_uchar4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ void st4(int8_t* p, int4 v) { *(char4*)p = make_char4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ void st4(uint16_t* p, int4 v) { *(ushort4*)p = make_ushort4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ void st4(int16_t* p, int4 v) { *(short4*)p = make_short4(v.x, v.y, v.z, v.w); }

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
// =============================================================================
#define DWT_TW 128
#define DWT_TH 32
#define DWT_LW (DWT_TW + 3)
#define DWT_LH (DWT_TH + 3)

__device__ __forceinline__ int mirror(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {   // at most one reflection for halo <= 2 unless n tiny
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

__global__ __launch_bounds__(256) void k_dwt53_fwd_level(const int32_t* __restrict__ src, uint32_t sstride,
                                                         int32_t* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h, GkTiles tb) {
    __shared__ int32_t T[DWT_LH][DWT_LW + 1];
    src += tb.offset(blockIdx.z, sstride); dst += tb.offset(blockIdx.z, dstride);
    const int x0 = blockIdx.x * DWT_TW, y0 = blockIdx.y * DWT_TH;
    const int tid = threadIdx.x;
    // 4 waves x 64 lanes: lane tx walks columns tx, tx+64, tx+128 of rows ty, ty+4, ... (no
    // index division: the level is bound by instruction count before HBM)
    const int tx = tid & 63, ty = tid >> 6;
    // load rows y0-2 .. y0+TH, cols x0-2 .. x0+TW (mirrored at the resolution border)
    if (x0 >= 2 && y0 >= 2 && x0 + DWT_TW < (int)w && y0 + DWT_TH < (int)h) {   // interior tile
        const int32_t* s0 = src + (size_t)(y0 - 2) * sstride + (x0 - 2);
        for (int ly = ty; ly < DWT_LH; ly += 4) {
            const int32_t* sr = s0 + (size_t)ly * sstride;
            T[ly][tx] = sr[tx];
            T[ly][tx + 64] = sr[tx + 64];
        }
        for (int i = tid; i < 3 * DWT_LH; i += 256) {   // columns 128..130
            const int ly = i / 3, lx = 128 + i % 3;
            T[ly][lx] = s0[(size_t)ly * sstride + lx];
        }
    } else {
        for (int i = tid; i < DWT_LH * DWT_LW; i += 256) {
            int ly = i / DWT_LW, lx = i % DWT_LW;
            int gy = mirror(y0 - 2 + ly, (int)h), gx = mirror(x0 - 2 + lx, (int)w);
            T[ly][lx] = src[(size_t)gy * sstride + gx];
        }
    }
    LDS_BARRIER();
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
    // scatter to quadrants: lane tx writes L and H sample k = tx of each row (coalesced rows)
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    const bool full = x0 + DWT_TW <= (int)w && y0 + DWT_TH <= (int)h;
    for (int ry = ty; ry < DWT_TH; ry += 4) {
        const int gy = y0 + ry;
        if (!full && gy >= (int)h) break;
        const int oy = ((gy & 1) == 0) ? (gy >> 1) : (snh + (gy >> 1));
        int32_t* drow = dst + (size_t)oy * dstride;
        const int gxl = x0 + 2 * tx;
        if (full || gxl < (int)w) drow[gxl >> 1] = T[ry + 2][2 + 2 * tx];
        if (full || gxl + 1 < (int)w) drow[snw + (gxl >> 1)] = T[ry + 2][3 + 2 * tx];
    }
}

// Inverse 5/3 level (WaveletReverse.cpp:802-879): horizontal then vertical,
// on the interleaved signal with symmetric extension.  Output tile rows
// y0..y0+TH-1; needs interleaved rows y0-1..y0+TH+1 and cols x0-1..x0+TW+1.
#define IDWT_LW (DWT_TW + 3)
#define IDWT_LH (DWT_TH + 3)
__global__ __launch_bounds__(256) void k_dwt53_inv_level(const int32_t* __restrict__ src, uint32_t sstride,
                                                         int32_t* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h, GkTiles tb) {
    __shared__ int32_t T[IDWT_LH][IDWT_LW + 1];
    src += tb.offset(blockIdx.z, sstride); dst += tb.offset(blockIdx.z, dstride);
    const int x0 = blockIdx.x * DWT_TW, y0 = blockIdx.y * DWT_TH;
    const int tid = threadIdx.x;
    const int tx = tid & 63, ty = tid >> 6;   // as in the forward level
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    if (x0 >= 1 && y0 >= 1 && x0 + DWT_TW + 1 < (int)w && y0 + DWT_TH + 1 < (int)h) {   // interior tile
        // interleaved column gx = x0 - 1 + lx: odd lx <=> even gx (L sample x0/2 + k, lx = 1 + 2k),
        // even lx <=> odd gx (H sample x0/2 - 1 + k, lx = 2k); both reads are contiguous
        for (int ly = ty; ly < IDWT_LH; ly += 4) {
            const int gy = y0 - 1 + ly;
            const int sy = (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1);
            const int32_t* sr = src + (size_t)sy * sstride;
            T[ly][1 + 2 * tx] = sr[(x0 >> 1) + tx];
            T[ly][2 * tx] = sr[snw + (x0 >> 1) - 1 + tx];
        }
        for (int i = tid; i < 3 * IDWT_LH; i += 256) {   // lx 128 (H), 129 (L), 130 (H)
            const int ly = i / 3, j = i % 3, gy = y0 - 1 + ly;
            const int sy = (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1);
            const int32_t* sr = src + (size_t)sy * sstride;
            T[ly][128 + j] = (j == 1) ? sr[(x0 >> 1) + 64] : sr[snw + (x0 >> 1) + 63 + (j >> 1)];
        }
    } else {
        for (int i = tid; i < IDWT_LH * IDWT_LW; i += 256) {
            int ly = i / IDWT_LW, lx = i % IDWT_LW;
            int gy = mirror(y0 - 1 + ly, (int)h), gx = mirror(x0 - 1 + lx, (int)w);
            int sy = (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1);
            int sx = (gx & 1) ? (snw + (gx >> 1)) : (gx >> 1);
            T[ly][lx] = src[(size_t)sy * sstride + sx];
        }
    }
    LDS_BARRIER();
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
    const bool full = x0 + DWT_TW <= (int)w && y0 + DWT_TH <= (int)h;
    for (int ry = ty; ry < DWT_TH; ry += 4) {
        const int gy = y0 + ry;
        if (!full && gy >= (int)h) break;
        int32_t* drow = dst + (size_t)gy * dstride + x0;
        for (int c = tx; c < DWT_TW; c += 64)
            if (full || x0 + c < (int)w) drow[c] = T[ry + 1][c + 1];
    }
}

// =============================================================================
// Byte gather for codestream assembly and decode staging.
// seg: (src_off, dst_off, len) triples; one wave per segment.
// =============================================================================
__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                const uint64_t* __restrict__ seg, uint32_t nseg) {
    uint32_t s = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= nseg) return;
    uint64_t so = seg[3 * s], d = seg[3 * s + 1], n = seg[3 * s + 2];
    const int lane = threadIdx.x & 63;
    for (uint64_t i = lane; i < n; i += 64) dst[d + i] = src[so + i];
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
    dim3 grid((w + 1023) / 1024, h);
    const int vec = vec_ok(gk_sample_size(stype), r, g, b, sin, 4, y, u, v, sout);
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_rct_fwd<T>, grid, dim3(256), 0, st, (const T*)r, (const T*)g, (const T*)b, sin, y, u, v,
                           sout, w, h, shift, vec))
}
void gk_launch_dc_fwd(hipStream_t st, int stype, const void* in, uint32_t sin, int32_t* out, uint32_t sout, uint32_t w,
                      uint32_t h, int32_t shift) {
    dim3 grid((w + 255) / 256, h);
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_fwd<T>, grid, dim3(256), 0, st, (const T*)in, sin, out, sout, w, h, shift))
}
void gk_launch_rct_inv_dc(hipStream_t st, const int32_t* y, const int32_t* u, const int32_t* v, uint32_t sin, int stype,
                          void* r, void* g, void* b, uint32_t sout, uint32_t w, uint32_t h, int32_t shift,
                          int32_t mn, int32_t mx) {
    dim3 grid((w + 1023) / 1024, h);
    const int vec = vec_ok(4, y, u, v, sin, gk_sample_size(stype), r, g, b, sout);
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_rct_inv_dc<T>, grid, dim3(256), 0, st, y, u, v, sin, (T*)r, (T*)g, (T*)b, sout, w, h, shift,
                           mn, mx, vec))
}
void gk_launch_dc_inv(hipStream_t st, const int32_t* in, uint32_t sin, int stype, void* out, uint32_t sout, uint32_t w,
                      uint32_t h, int32_t shift, int32_t mn, int32_t mx) {
    dim3 grid((w + 255) / 256, h);
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_inv<T>, grid, dim3(256), 0, st, in, sin, (T*)out, sout, w, h, shift, mn, mx))
}
void gk_launch_dwt53_fwd(hipStream_t st, const int32_t* src, uint32_t sstride, int32_t* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb) {
    dim3 grid((w + DWT_TW - 1) / DWT_TW, (h + DWT_TH - 1) / DWT_TH, tb.count());
    hipLaunchKernelGGL(k_dwt53_fwd_level, grid, dim3(256), 0, st, src, sstride, dst, dstride, w, h, tb);
}
void gk_launch_dwt53_inv(hipStream_t st, const int32_t* src, uint32_t sstride, int32_t* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb) {
    dim3 grid((w + DWT_TW - 1) / DWT_TW, (h + DWT_TH - 1) / DWT_TH, tb.count());
    hipLaunchKernelGGL(k_dwt53_inv_level, grid, dim3(256), 0, st, src, sstride, dst, dstride, w, h, tb);
}
void gk_launch_gather(hipStream_t st, const uint8_t* src, uint8_t* dst, const uint64_t* seg, uint32_t nseg) {
    if (!nseg) return;
    hipLaunchKernelGGL(k_gather, dim3((nseg + 3) / 4), dim3(256), 0, st, src, dst, seg, nseg);
}
