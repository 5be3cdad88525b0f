// gk_dwt97.hip — irreversible path kernels for gfx950: ICT, 9/7 DWT (fwd/inv),
// and the irreversible DC/clamp stages.
//
// Bit-exactness: every lifting step is x_i = x_i + (x_{i-1} + x_{i+1}) * c with
// no FMA contraction, the order Grok evaluates it in (dwt97::encode_step2 and
// grk_v8dwt_encode_step2, WaveletFwd.cpp:135-163, 370-398; decompress_step2_97,
// WaveletReverse.cpp:964-1022), so the GPU transform reproduces Grok's float
// results bit for bit.  Boundaries use whole-sample symmetric extension of the
// input (identical values to Grok's "2 * neighbour" edge rule).
//
// Tiling: one launch per decomposition level; a 256-thread workgroup owns a
// 128 x 32 output tile, loads it with a 4-sample halo on every side into LDS,
// runs the vertical then the horizontal lifting (forward) or horizontal then
// vertical (inverse) in LDS, and scatters to the four Mallat quadrants.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"
#include "gk_xcd.h"

#pragma clang fp contract(off)

#define T97_W 128
#define T97_H 32
#define T97_HALO 4
#define T97_LW (T97_W + 2 * T97_HALO)
#define T97_LH (T97_H + 2 * T97_HALO)

// WaveletFwd.cpp:39-44 (float constants; invK computed in double then rounded)
#define F97_A (-1.586134342f)
#define F97_B (-0.052980118f)
#define F97_G (0.882911075f)
#define F97_D (0.443506852f)
#define F97_K (1.230174105f)
#define F97_INVK ((float)(1.0 / 1.230174105))
// WaveletReverse.cpp:365-371
#define I97_A (1.586134342f)
#define I97_B (0.052980118f)
#define I97_G (-0.882911075f)
#define I97_D (-0.443506852f)
#define I97_TWO_INVK (1.625732422f)

__device__ __forceinline__ int mirror97(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

// =============================================================================
// DC shift + ICT forward (mct.cpp:147-219 CompressIrrev; TileProcessor.cpp:506-535).
// Output: float written over int32 storage, as in Grok.
// =============================================================================
template <class TI>
__global__ __launch_bounds__(256) void k_dc_ict_fwd(const TI* __restrict__ r_in, const TI* __restrict__ g_in,
                                                    const TI* __restrict__ b_in, uint32_t sin,
                                                    float* __restrict__ y_out, float* __restrict__ u_out,
                                                    float* __restrict__ v_out, uint32_t sout, uint32_t w, uint32_t h,
                                                    int32_t shift) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= w || y >= h) return;
    const float a_r = 0.299f, a_g = 0.587f, a_b = 0.114f;
    const float cb = 0.5f / (1.0f - a_b), cr = 0.5f / (1.0f - a_r);
    const size_t i = (size_t)y * sin + x, o = (size_t)y * sout + x;
    float r = (float)((int32_t)r_in[i] - shift), g = (float)((int32_t)g_in[i] - shift), b = (float)((int32_t)b_in[i] - shift);
    float t0 = a_r * r, t1 = a_g * g, t2 = a_b * b;
    float Y = (t0 + t1) + t2;
    y_out[o] = Y;
    u_out[o] = cb * (b - Y);
    v_out[o] = cr * (r - Y);
}

// DC shift to float without MCT (the standard behaviour; Grok's mono 9/7 path
// multiplies by 2048 and reinterprets — R-BUG-1, not reproduced).
template <class TI>
__global__ __launch_bounds__(256) void k_dc_fwd_f(const TI* __restrict__ in, uint32_t sin, float* __restrict__ out,
                                                  uint32_t sout, uint32_t w, uint32_t h, int32_t shift) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= w || y >= h) return;
    out[(size_t)y * sout + x] = (float)((int32_t)in[(size_t)y * sin + x] - shift);
}

// Inverse ICT + DC shift + clamp (mct.cpp:284-364 DecompressIrrev, lrintf rounding).
template <class TO>
__global__ __launch_bounds__(256) void k_ict_inv_dc(const float* __restrict__ y_in, const float* __restrict__ u_in,
                                                    const float* __restrict__ v_in, uint32_t sin,
                                                    TO* __restrict__ r_out, TO* __restrict__ g_out,
                                                    TO* __restrict__ b_out, uint32_t sout, uint32_t w, uint32_t h,
                                                    int32_t shift, int32_t mn, int32_t mx) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= w || y >= h) return;
    const size_t i = (size_t)y * sin + x, o = (size_t)y * sout + x;
    float Y = y_in[i], U = u_in[i], V = v_in[i];
    float R = Y + 1.402f * V;
    float G = (Y - 0.34413f * U) - 0.71414f * V;
    float B = Y + 1.772f * U;
    auto cl = [&](float f) { int32_t v = (int32_t)rintf(f) + shift; return (TO)(v < mn ? mn : (v > mx ? mx : v)); };
    r_out[o] = cl(R); g_out[o] = cl(G); b_out[o] = cl(B);
}

template <class TO>
__global__ __launch_bounds__(256) void k_dc_inv_f(const float* __restrict__ in, uint32_t sin, TO* __restrict__ out,
                                                  uint32_t sout, uint32_t w, uint32_t h, int32_t shift, int32_t mn,
                                                  int32_t mx) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= w || y >= h) return;
    int32_t v = (int32_t)rintf(in[(size_t)y * sin + x]) + shift;
    out[(size_t)y * sout + x] = (TO)(v < mn ? mn : (v > mx ? mx : v));
}

// =============================================================================
// Forward 9/7, one level (WaveletFwd.cpp:964-1025): vertical then horizontal.
// Components in grid.z (GkComps); level 1 fused with DC + ICT (k_dwt97_fwd_l1) and the
// last inverse level with the inverse ICT + DC + clamp (k_dwt97_inv_l1), as for the 5/3.
// =============================================================================
typedef float Lds97[T97_LH][T97_LW + 1];

// f(ly, lx, gy, gx): the sample at mirrored input position (gy, gx) into LDS (ly, lx)
template <class F>
__device__ __forceinline__ void fwd97_fill(int x0, int y0, int w, int h, int tid, F f) {
    for (int i = tid; i < T97_LH * T97_LW; i += 256) {
        const int ly = i / T97_LW, lx = i % T97_LW;
        f(ly, lx, mirror97(y0 - T97_HALO + ly, h), mirror97(x0 - T97_HALO + lx, w));
    }
}

__device__ __forceinline__ void fwd97_lift(Lds97& T, int w, int h, int tid) {
    // local row ly <-> global y0 - 4 + ly; parity of global y == parity of ly (y0 even)
    if (h > 1) {
        const float cs[4] = {F97_A, F97_B, F97_G, F97_D};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int par = (s & 1) ? 0 : 1;          // alpha/gamma update odd rows, beta/delta even rows
            const int lo = 1 + s, hi = T97_LH - 2 - s;  // rows with both neighbours still valid
            const int first = lo + ((lo & 1) != par);
            const int nrows = first > hi ? 0 : (hi - first) / 2 + 1;
            for (int i = tid; i < nrows * T97_LW; i += 256) {
                int ly = first + 2 * (i / T97_LW), lx = i % T97_LW;
                float t = (T[ly - 1][lx] + T[ly + 1][lx]) * cs[s];
                T[ly][lx] = T[ly][lx] + t;
            }
            __syncthreads();
        }
        for (int i = tid; i < T97_H * T97_LW; i += 256) {
            int ly = T97_HALO + i / T97_LW, lx = i % T97_LW;
            T[ly][lx] = T[ly][lx] * ((ly & 1) ? F97_K : F97_INVK);
        }
        __syncthreads();
    }
    if (w > 1) {
        const float cs[4] = {F97_A, F97_B, F97_G, F97_D};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int par = (s & 1) ? 0 : 1;
            const int lo = 1 + s, hi = T97_LW - 2 - s;
            const int first = lo + ((lo & 1) != par);
            const int ncols = first > hi ? 0 : (hi - first) / 2 + 1;
            for (int i = tid; i < T97_H * ncols; i += 256) {
                int ly = T97_HALO + i / ncols, lx = first + 2 * (i % ncols);
                float t = (T[ly][lx - 1] + T[ly][lx + 1]) * cs[s];
                T[ly][lx] = T[ly][lx] + t;
            }
            __syncthreads();
        }
        for (int i = tid; i < T97_H * T97_W; i += 256) {
            int ly = T97_HALO + i / T97_W, lx = T97_HALO + i % T97_W;
            T[ly][lx] = T[ly][lx] * ((lx & 1) ? F97_K : F97_INVK);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ void fwd97_store(const Lds97& T, float* __restrict__ dst, uint32_t dstride, int x0, int y0,
                                            int w, int h, int tid) {
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    for (int i = tid; i < T97_H * T97_W; i += 256) {
        int ry = i / T97_W, rx = i % T97_W;
        int q = rx / (T97_W / 2), k = rx % (T97_W / 2);
        int gx = x0 + 2 * k + q, gy = y0 + ry;
        if (gx >= w || gy >= h) continue;
        float v = T[ry + T97_HALO][2 * k + q + T97_HALO];
        int ox = (q == 0) ? (gx >> 1) : (snw + (gx >> 1));
        int oy = ((gy & 1) == 0) ? (gy >> 1) : (snh + (gy >> 1));
        dst[(size_t)oy * dstride + ox] = v;
    }
}

__global__ __launch_bounds__(256) void k_dwt97_fwd_level(const float* __restrict__ src, uint32_t sstride,
                                                         float* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h, GkTiles tb, GkComps cs) {
    __shared__ Lds97 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z % tb.count(), comp = bi.z / tb.count();
    src += tb.offset(tile, sstride) + comp * cs.cstride;
    dst += tb.offset(tile, dstride) + comp * cs.cstride;
    const int x0 = bi.x * T97_W, y0 = bi.y * T97_H, tid = threadIdx.x;
    fwd97_fill(x0, y0, (int)w, (int)h, tid,
               [&](int ly, int lx, int gy, int gx) { T[ly][lx] = src[(size_t)gy * sstride + gx]; });
    __syncthreads();
    fwd97_lift(T, (int)w, (int)h, tid);
    fwd97_store(T, dst, dstride, x0, y0, (int)w, (int)h, tid);
}

// Level 1 from the caller's planes: DC shift and, for NC = 3, the ICT (mct.cpp:147-219) on load.
// One LDS tile: Y goes first while each thread keeps U and V of its positions in registers
// (22 slots = ceil(40 x 136 / 256)), then U, then V (as k_dwt53_fwd_l1).
#define L97_SLOTS 22
template <class F>   // f(slot, ly, lx, gy, gx) over fwd97_fill's positions
__device__ __forceinline__ void fwd97_fill_slots(int x0, int y0, int w, int h, int tid, F f) {
#pragma unroll
    for (int k = 0; k < L97_SLOTS; ++k) {
        const int i = tid + 256 * k;
        if (i < T97_LH * T97_LW) {
            const int ly = i / T97_LW, lx = i % T97_LW;
            f(k, ly, lx, mirror97(y0 - T97_HALO + ly, h), mirror97(x0 - T97_HALO + lx, w));
        }
    }
}

template <class TI, int NC>
__global__ __launch_bounds__(256) void k_dwt97_fwd_l1(GkPtr3 in, uint32_t sin, float* __restrict__ dst, uint64_t cstride,
                                                      uint32_t dstride, uint32_t w, uint32_t h, GkTiles tb,
                                                      int32_t shift) {
    __shared__ Lds97 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z;
    const uint64_t io = tb.offset(tile, sin);
    const TI* p0 = (const TI*)in.p[0] + io;
    const TI* p1 = (const TI*)in.p[NC == 3 ? 1 : 0] + io;
    const TI* p2 = (const TI*)in.p[NC == 3 ? 2 : 0] + io;
    dst += tb.offset(tile, dstride);
    const int x0 = bi.x * T97_W, y0 = bi.y * T97_H, tid = threadIdx.x;
    float U[L97_SLOTS], V[L97_SLOTS];
    fwd97_fill_slots(x0, y0, (int)w, (int)h, tid, [&](int k, int ly, int lx, int gy, int gx) {
        const size_t i = (size_t)gy * sin + gx;
        if (NC == 3) {
            const float a_r = 0.299f, a_g = 0.587f, a_b = 0.114f;
            const float cb = 0.5f / (1.0f - a_b), cr = 0.5f / (1.0f - a_r);
            const float r = (float)((int32_t)p0[i] - shift), g = (float)((int32_t)p1[i] - shift),
                        b = (float)((int32_t)p2[i] - shift);
            const float t0 = a_r * r, t1 = a_g * g, t2 = a_b * b;
            const float Y = (t0 + t1) + t2;
            T[ly][lx] = Y;
            U[k] = cb * (b - Y);
            V[k] = cr * (r - Y);
        } else {
            T[ly][lx] = (float)((int32_t)p0[i] - shift);
        }
    });
    __syncthreads();
    fwd97_lift(T, (int)w, (int)h, tid);
    fwd97_store(T, dst, dstride, x0, y0, (int)w, (int)h, tid);
    if (NC == 3) {
#pragma unroll
        for (int c = 1; c < 3; ++c) {
            __syncthreads();
            fwd97_fill_slots(x0, y0, (int)w, (int)h, tid,
                             [&](int k, int ly, int lx, int, int) { T[ly][lx] = c == 1 ? U[k] : V[k]; });
            __syncthreads();
            fwd97_lift(T, (int)w, (int)h, tid);
            fwd97_store(T, dst + c * cstride, dstride, x0, y0, (int)w, (int)h, tid);
        }
    }
}

// =============================================================================
// Inverse 9/7, one level (WaveletReverse.cpp:1010-1022, 1272-1351):
// horizontal then vertical, on the interleaved signal.
// =============================================================================
template <class F>
__device__ __forceinline__ void inv97_fill(int x0, int y0, int w, int h, int tid, F f) {
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    for (int i = tid; i < T97_LH * T97_LW; i += 256) {
        int ly = i / T97_LW, lx = i % T97_LW;
        int gy = mirror97(y0 - T97_HALO + ly, h), gx = mirror97(x0 - T97_HALO + lx, w);
        f(ly, lx, (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1), (gx & 1) ? (snw + (gx >> 1)) : (gx >> 1));
    }
}

__device__ __forceinline__ void inv97_lift(Lds97& T, int w, int h, int tid) {
    const float cs[4] = {I97_D, I97_G, I97_B, I97_A};
    if (w > 1) {
        for (int i = tid; i < T97_LH * T97_LW; i += 256) {
            int ly = i / T97_LW, lx = i % T97_LW;
            T[ly][lx] = T[ly][lx] * ((lx & 1) ? I97_TWO_INVK : F97_K);
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int par = (s & 1) ? 1 : 0;            // delta/beta on even samples, gamma/alpha on odd
            const int lo = 1 + s, hi = T97_LW - 2 - s;
            const int first = lo + ((lo & 1) != par);
            const int ncols = first > hi ? 0 : (hi - first) / 2 + 1;
            for (int i = tid; i < T97_LH * ncols; i += 256) {
                int ly = i / ncols, lx = first + 2 * (i % ncols);
                float t = (T[ly][lx - 1] + T[ly][lx + 1]) * cs[s];
                T[ly][lx] = T[ly][lx] + t;
            }
            __syncthreads();
        }
    }
    if (h > 1) {
        for (int i = tid; i < T97_LH * T97_W; i += 256) {
            int ly = i / T97_W, lx = T97_HALO + i % T97_W;
            T[ly][lx] = T[ly][lx] * ((ly & 1) ? I97_TWO_INVK : F97_K);
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int par = (s & 1) ? 1 : 0;
            const int lo = 1 + s, hi = T97_LH - 2 - s;
            const int first = lo + ((lo & 1) != par);
            const int nrows = first > hi ? 0 : (hi - first) / 2 + 1;
            for (int i = tid; i < nrows * T97_W; i += 256) {
                int ly = first + 2 * (i / T97_W), lx = T97_HALO + i % T97_W;
                float t = (T[ly - 1][lx] + T[ly + 1][lx]) * cs[s];
                T[ly][lx] = T[ly][lx] + t;
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(256) void k_dwt97_inv_level(const float* __restrict__ src, uint32_t sstride,
                                                         float* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h, GkTiles tb, GkComps cs) {
    __shared__ Lds97 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z % tb.count(), comp = bi.z / tb.count();
    src += tb.offset(tile, sstride) + comp * cs.cstride;
    dst += tb.offset(tile, dstride) + comp * cs.cstride;
    const int x0 = bi.x * T97_W, y0 = bi.y * T97_H, tid = threadIdx.x;
    inv97_fill(x0, y0, (int)w, (int)h, tid,
               [&](int ly, int lx, int sy, int sx) { T[ly][lx] = src[(size_t)sy * sstride + sx]; });
    __syncthreads();
    inv97_lift(T, (int)w, (int)h, tid);
    for (int i = tid; i < T97_H * T97_W; i += 256) {
        int ry = i / T97_W, rx = i % T97_W;
        int gx = x0 + rx, gy = y0 + ry;
        if (gx >= (int)w || gy >= (int)h) continue;
        dst[(size_t)gy * dstride + gx] = T[ry + T97_HALO][rx + T97_HALO];
    }
}

// Last inverse level into the caller's planes: inverse ICT for NC = 3 (mct.cpp:284-364,
// lrintf rounding), DC shift and clamp, only inside the output window (GkWin).  One LDS
// tile; the Y and U results of each thread's 16 output samples wait in registers.
template <class TO, int NC>
__global__ __launch_bounds__(256) void k_dwt97_inv_l1(const float* __restrict__ src, uint64_t cstride, uint32_t sstride,
                                                      GkPtr3 out, uint32_t ostride, GkWin win, uint32_t w, uint32_t h,
                                                      GkTiles tb, int32_t shift, int32_t mn, int32_t mx) {
    __shared__ Lds97 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z;
    src += tb.offset(tile, sstride);
    int32_t ox, oy;
    tb.origin(tile, ox, oy);
    const int x0 = bi.x * T97_W, y0 = bi.y * T97_H, tid = threadIdx.x;
    float R0[16], R1[16];   // sample i = tid + 256 k of the 32 x 128 output tile
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (c) __syncthreads();
        const float* sc = src + c * cstride;
        inv97_fill(x0, y0, (int)w, (int)h, tid,
                   [&](int ly, int lx, int sy, int sx) { T[ly][lx] = sc[(size_t)sy * sstride + sx]; });
        __syncthreads();
        inv97_lift(T, (int)w, (int)h, tid);
        if (c + 1 < NC) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int i = tid + 256 * k;
                (c == 0 ? R0 : R1)[k] = T[i / T97_W + T97_HALO][i % T97_W + T97_HALO];
            }
        }
    }
    TO* o0 = (TO*)out.p[0];
    TO* o1 = (TO*)out.p[NC == 3 ? 1 : 0];
    TO* o2 = (TO*)out.p[NC == 3 ? 2 : 0];
    auto cl = [&](float f) { int32_t v = (int32_t)rintf(f) + shift; return (TO)(v < mn ? mn : (v > mx ? mx : v)); };
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int i = tid + 256 * k;
        const int ry = i / T97_W, rx = i % T97_W;
        const int gx = x0 + rx, gy = y0 + ry, X = ox + gx, Y = oy + gy;
        if (gx >= (int)w || gy >= (int)h || X < win.x0 || X >= win.x1 || Y < win.y0 || Y >= win.y1) continue;
        const size_t o = (size_t)(Y - win.y0) * ostride + (X - win.x0);
        const float last = T[ry + T97_HALO][rx + T97_HALO];
        if (NC == 3) {
            const float Yv = R0[k], U = R1[k], V = last;
            const float R = Yv + 1.402f * V;
            const float G = (Yv - 0.34413f * U) - 0.71414f * V;
            const float B = Yv + 1.772f * U;
            o0[o] = cl(R); o1[o] = cl(G); o2[o] = cl(B);
        } else {
            o0[o] = cl(last);
        }
    }
}

#include "gk_launch.h"

void gk_launch_dc_ict_fwd(hipStream_t st, int stype, const void* r, const void* g, const void* b, uint32_t sin, float* y,
                          float* u, float* v, uint32_t sout, uint32_t w, uint32_t h, int32_t shift) {
    if (!w || !h) return;   // an empty region (a resolution of zero width or height): no launch
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_ict_fwd<T>, dim3((w + 255) / 256, h), dim3(256), 0, st, (const T*)r, (const T*)g,
                           (const T*)b, sin, y, u, v, sout, w, h, shift))
}
void gk_launch_dc_fwd_f(hipStream_t st, int stype, const void* in, uint32_t sin, float* out, uint32_t sout, uint32_t w,
                        uint32_t h, int32_t shift) {
    if (!w || !h) return;   // an empty region (a resolution of zero width or height): no launch
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_fwd_f<T>, dim3((w + 255) / 256, h), dim3(256), 0, st, (const T*)in, sin, out, sout, w, h,
                           shift))
}
void gk_launch_ict_inv_dc(hipStream_t st, const float* y, const float* u, const float* v, uint32_t sin, int stype, void* r,
                          void* g, void* b, uint32_t sout, uint32_t w, uint32_t h, int32_t shift, int32_t mn,
                          int32_t mx) {
    if (!w || !h) return;   // an empty region (a resolution of zero width or height): no launch
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_ict_inv_dc<T>, dim3((w + 255) / 256, h), dim3(256), 0, st, y, u, v, sin, (T*)r, (T*)g, (T*)b,
                           sout, w, h, shift, mn, mx))
}
void gk_launch_dc_inv_f(hipStream_t st, const float* in, uint32_t sin, int stype, void* out, uint32_t sout, uint32_t w,
                        uint32_t h, int32_t shift, int32_t mn, int32_t mx) {
    if (!w || !h) return;   // an empty region (a resolution of zero width or height): no launch
    GK_SAMPLE_DISPATCH(stype, T,
        hipLaunchKernelGGL(k_dc_inv_f<T>, dim3((w + 255) / 256, h), dim3(256), 0, st, in, sin, (T*)out, sout, w, h, shift,
                           mn, mx))
}
static uint32_t comps_in_grid97(GkTiles tb, GkComps cs) { return tb.count() * cs.n <= 65535u ? cs.n : 1u; }
void gk_launch_dwt97_fwd(hipStream_t st, const float* src, uint32_t sstride, float* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb, GkComps cs) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    const uint32_t ng = comps_in_grid97(tb, cs);
    for (uint32_t c = 0; c < cs.n; c += ng) {
        GkComps g = cs; g.n = ng;
        dim3 grid((w + T97_W - 1) / T97_W, (h + T97_H - 1) / T97_H, tb.count() * ng);
        hipLaunchKernelGGL(k_dwt97_fwd_level, grid, dim3(256), 0, st, src + c * cs.cstride, sstride, dst + c * cs.cstride,
                           dstride, w, h, tb, g);
    }
}
void gk_launch_dwt97_inv(hipStream_t st, const float* src, uint32_t sstride, float* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb, GkComps cs) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    const uint32_t ng = comps_in_grid97(tb, cs);
    for (uint32_t c = 0; c < cs.n; c += ng) {
        GkComps g = cs; g.n = ng;
        dim3 grid((w + T97_W - 1) / T97_W, (h + T97_H - 1) / T97_H, tb.count() * ng);
        hipLaunchKernelGGL(k_dwt97_inv_level, grid, dim3(256), 0, st, src + c * cs.cstride, sstride, dst + c * cs.cstride,
                           dstride, w, h, tb, g);
    }
}
void gk_launch_dwt97_fwd_l1(hipStream_t st, int stype, int nc, GkPtr3 in, uint32_t sin, float* dst, uint64_t cstride,
                            uint32_t dstride, uint32_t w, uint32_t h, GkTiles tb, int32_t shift) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + T97_W - 1) / T97_W, (h + T97_H - 1) / T97_H, tb.count());
    if (nc == 3)
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt97_fwd_l1<T, 3>), grid, dim3(256), 0, st, in, sin, dst,
                                                        cstride, dstride, w, h, tb, shift))
    else
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt97_fwd_l1<T, 1>), grid, dim3(256), 0, st, in, sin, dst,
                                                        cstride, dstride, w, h, tb, shift))
}
void gk_launch_dwt97_inv_l1(hipStream_t st, int stype, int nc, const float* src, uint64_t cstride, uint32_t sstride,
                            GkPtr3 out, uint32_t ostride, GkWin win, uint32_t w, uint32_t h, GkTiles tb, int32_t shift,
                            int32_t mn, int32_t mx) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + T97_W - 1) / T97_W, (h + T97_H - 1) / T97_H, tb.count());
    if (nc == 3)
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt97_inv_l1<T, 3>), grid, dim3(256), 0, st, src, cstride,
                                                        sstride, out, ostride, win, w, h, tb, shift, mn, mx))
    else
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt97_inv_l1<T, 1>), grid, dim3(256), 0, st, src, cstride,
                                                        sstride, out, ostride, win, w, h, tb, shift, mn, mx))
}
