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
#include "gk_vec.h"

#pragma clang fp contract(off)

#define T97_W 128
#define T97_H 32
#define T97_HALO 4
#define T97_LW (T97_W + 2 * T97_HALO)   // 136
#define T97_LH (T97_H + 2 * T97_HALO)   // 40

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
//
// The tile is 136 x 40 samples in LDS (a 4-sample halo around the 128 x 32 outputs).  Work is
// mapped without index division: a wave takes rows (ty, ty + 4, ...), its lanes columns tx and
// tx + 64, and the few halo columns / rows past 64 updates go in one extra pass.  The scalings
// are folded into neighbouring passes, multiplying each value exactly where Grok's separate
// pass would have (the same float products, so the results are unchanged):
//  * forward: the vertical K / 1/K of a row into horizontal steps 0 and 1 (every value those
//    steps read is scaled as it is read until step 1 has written it), the horizontal one into
//    the store;
//  * inverse: the horizontal K / 2/K into the fill, the vertical one into vertical steps 0
//    and 1 in the same way.
// Interior tiles (no mirrored sample) read and write the caller's planes four samples per lane.
// =============================================================================
typedef float Lds97[T97_LH][T97_LW + 1];

// a tile whose 128 columns lie inside the resolution takes the lane-mapped paths (rows and
// halo columns mirrored where they fall outside: a tile-grid border); a last, partial tile
// column the general per-position one
__device__ __forceinline__ bool fullw97(int x0, int w) { return x0 + T97_W <= w; }

// f(ly, lx, gy, gx): the sample at mirrored input position (gy, gx) into LDS (ly, lx) (partial tiles)
template <class F>
__device__ __forceinline__ void fwd97_fill(int x0, int y0, int w, int h, int tid, F f) {
    for (int i = tid; i < T97_LH * T97_LW; i += 256) {
        const int ly = i / T97_LW, lx = i % T97_LW;
        f(ly, lx, mirror97(y0 - T97_HALO + ly, h), mirror97(x0 - T97_HALO + lx, w));
    }
}
// full-width tile: LDS columns 4..131 by the lanes, halo columns 0..3 / 132..135 in one pass
template <class F>
__device__ __forceinline__ void fwd97_fill_inner(int x0, int y0, int w, int h, int tid, F f) {
    const int tx = tid & 63, ty = tid >> 6;
    for (int ly = ty; ly < T97_LH; ly += 4) {
        const int gy = mirror97(y0 - T97_HALO + ly, h);
        f(ly, 4 + tx, gy, x0 + tx);
        f(ly, 68 + tx, gy, x0 + 64 + tx);
    }
    for (int i = tid; i < 8 * T97_LH; i += 256) {
        const int ly = i >> 3, j = i & 7, lx = j < 4 ? j : 128 + j;
        f(ly, lx, mirror97(y0 - T97_HALO + ly, h), mirror97(x0 - T97_HALO + lx, w));
    }
}

__device__ __forceinline__ void fwd97_lift(Lds97& T, int w, int h, int tid) {
    const int tx = tid & 63, ty = tid >> 6;
    // local row ly <-> global y0 - 4 + ly; parity of global y == parity of ly (y0 even)
    if (h > 1) {
        // step s (alpha, beta, gamma, delta) updates rows 1 + s, 3 + s, ... (19 - s rows) of every column
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float c = s == 0 ? F97_A : (s == 1 ? F97_B : (s == 2 ? F97_G : F97_D));
            const int first = 1 + s, nrows = 19 - s;
            auto upd = [&](int ly, int lx) {
                const float t = (T[ly - 1][lx] + T[ly + 1][lx]) * c;
                T[ly][lx] = T[ly][lx] + t;
            };
            for (int m = ty; m < nrows; m += 4) { upd(first + 2 * m, tx); upd(first + 2 * m, 64 + tx); }
            if (tid < nrows * 8) upd(first + 2 * (tid >> 3), 128 + (tid & 7));
            __syncthreads();
        }
        if (w <= 1) {   // no horizontal pass to fold the scaling into
            for (int i = tid; i < T97_H * T97_LW; i += 256) {
                const int ly = T97_HALO + i / T97_LW, lx = i % T97_LW;
                T[ly][lx] = T[ly][lx] * ((ly & 1) ? F97_K : F97_INVK);
            }
            __syncthreads();
        }
    }
    if (w > 1) {
        const bool vs = h > 1;   // the vertical scaling of rows 4..35 is still to apply
        // step s updates columns 1 + s, 3 + s, ... (67 - s columns) of the output rows 4..35
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float c = s == 0 ? F97_A : (s == 1 ? F97_B : (s == 2 ? F97_G : F97_D));
            const int first = 1 + s, e = 3 - s;   // e: columns past the lanes' 64
            auto upd = [&](int ly, int lx) {
                const float f = vs ? ((ly & 1) ? F97_K : F97_INVK) : 1.0f;
                if (s == 0 && vs) {   // nothing in the row is scaled yet
                    const float t = (T[ly][lx - 1] * f + T[ly][lx + 1] * f) * c;
                    T[ly][lx] = T[ly][lx] * f + t;
                } else if (s == 1 && vs) {   // the odd columns are (step 0 wrote them)
                    const float t = (T[ly][lx - 1] + T[ly][lx + 1]) * c;
                    T[ly][lx] = T[ly][lx] * f + t;
                } else {
                    const float t = (T[ly][lx - 1] + T[ly][lx + 1]) * c;
                    T[ly][lx] = T[ly][lx] + t;
                }
            };
            for (int ly = T97_HALO + ty; ly < T97_HALO + T97_H; ly += 4) upd(ly, first + 2 * tx);
            if (e && tid < T97_H * e) upd(T97_HALO + tid / e, first + 2 * (64 + tid % e));
            __syncthreads();
        }
    }
}

// the four Mallat quadrants; the horizontal scaling (K odd, 1/K even columns) on the way out
__device__ __forceinline__ void fwd97_store(const Lds97& T, float* __restrict__ dst, uint32_t dstride, int x0, int y0,
                                            int w, int h, int tid) {
    const int tx = tid & 63, ty = tid >> 6;
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    const float fl = w > 1 ? F97_INVK : 1.0f, fh = w > 1 ? F97_K : 1.0f;
    const int gx = x0 + 2 * tx;
    for (int ry = ty; ry < T97_H; ry += 4) {
        const int gy = y0 + ry;
        if (gy >= h) break;
        const int oy = ((gy & 1) == 0) ? (gy >> 1) : (snh + (gy >> 1));
        float* drow = dst + (size_t)oy * dstride;
        if (gx < w) drow[gx >> 1] = T[ry + T97_HALO][T97_HALO + 2 * tx] * fl;
        if (gx + 1 < w) drow[snw + (gx >> 1)] = T[ry + T97_HALO][T97_HALO + 1 + 2 * tx] * fh;
    }
}

// One level, cpw components per workgroup; full-width tiles prefetch the next component's input
// into registers while the current one lifts (as k_dwt53_fwd_level)
__global__ __launch_bounds__(256) void k_dwt97_fwd_level(const float* __restrict__ src, uint32_t sstride,
                                                         float* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h, GkTiles tb, GkComps cs, uint32_t cpw) {
    __shared__ Lds97 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z % tb.count(), c0 = bi.z / tb.count() * cpw, c1 = min(cs.n, c0 + cpw);
    src += tb.offset(tile, sstride);
    dst += tb.offset(tile, dstride);
    const int x0 = bi.x * T97_W, y0 = bi.y * T97_H, tid = threadIdx.x;
    const int tx = tid & 63, ty = tid >> 6;
    constexpr int PF_ROWS = (T97_LH + 3) / 4, PF_HALO = (8 * T97_LH + 255) / 256;
    float PF[2 * PF_ROWS + PF_HALO];
    const bool inner = fullw97(x0, (int)w);
    auto hlx = [](int i) { const int j = i & 7; return j < 4 ? j : 128 + j; };
    auto fetch = [&](const float* sc) {   // (fwd97_fill_inner's positions)
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < T97_LH) {
                const float* r = sc + (size_t)mirror97(y0 - T97_HALO + ly, (int)h) * sstride + x0 + tx;
                PF[2 * m] = r[0];
                PF[2 * m + 1] = r[64];
            }
        }
#pragma unroll
        for (int k = 0; k < PF_HALO; ++k) {
            const int i = tid + 256 * k;
            if (i < 8 * T97_LH)
                PF[2 * PF_ROWS + k] = sc[(size_t)mirror97(y0 - T97_HALO + (i >> 3), (int)h) * sstride +
                                         mirror97(x0 - T97_HALO + hlx(i), (int)w)];
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < T97_LH) { T[ly][4 + tx] = PF[2 * m]; T[ly][68 + tx] = PF[2 * m + 1]; }
        }
#pragma unroll
        for (int k = 0; k < PF_HALO; ++k) {
            const int i = tid + 256 * k;
            if (i < 8 * T97_LH) T[i >> 3][hlx(i)] = PF[2 * PF_ROWS + k];
        }
    };
    if (inner) fetch(src + c0 * cs.cstride);
    for (uint32_t c = c0; c < c1; ++c) {
        if (c != c0) __syncthreads();   // the previous component's stores have read the tile
        const float* sc = src + c * cs.cstride;
        if (inner) put();
        else fwd97_fill(x0, y0, (int)w, (int)h, tid,
                        [&](int ly, int lx, int gy, int gx) { T[ly][lx] = sc[(size_t)gy * sstride + gx]; });
        __syncthreads();
        if (inner && c + 1 < c1) fetch(sc + cs.cstride);
        fwd97_lift(T, (int)w, (int)h, tid);
        fwd97_store(T, dst + c * cs.cstride, dstride, x0, y0, (int)w, (int)h, tid);
    }
}

// Level 1 from the caller's planes: DC shift and, for NC = 3, the ICT (mct.cpp:147-219) on load.
// One LDS tile: Y goes first while each thread keeps U and V of its positions in registers,
// then U, then V (as k_dwt53_fwd_l1).  Interior tiles: six groups of four consecutive samples per
// thread (five of the 40 x 32 main groups, one of the 80 halo groups), one vector load per group
// and plane; edge tiles: 22 mirrored positions per thread.
#define L97_SLOTS 24
template <class F>   // f(slot, ly, lx, gy, gx): edge-tile positions, slot < 22
__device__ __forceinline__ void fwd97_fill_slots(int x0, int y0, int w, int h, int tid, F f) {
#pragma unroll
    for (int k = 0; k < 22; ++k) {
        const int i = tid + 256 * k;
        if (i < T97_LH * T97_LW) {
            const int ly = i / T97_LW, lx = i % T97_LW;
            f(k, ly, lx, mirror97(y0 - T97_HALO + ly, h), mirror97(x0 - T97_HALO + lx, w));
        }
    }
}
template <class F>   // f(group, ly, lx): interior groups of four positions (ly, lx .. lx + 3)
__device__ __forceinline__ void fwd97_groups(int tid, F f) {
#pragma unroll
    for (int g = 0; g < 6; ++g) {
        const int i = tid + 256 * g;
        if (g < 5) f(g, i >> 5, T97_HALO + 4 * (i & 31));
        else if (tid < 2 * T97_LH) f(g, tid >> 1, (tid & 1) ? T97_HALO + T97_W : 0);
    }
}

template <class TI, int NC>
__global__ __launch_bounds__(256) void k_dwt97_fwd_l1(GkPtr3 in, uint32_t sin, float* __restrict__ dst, uint64_t cstride,
                                                      uint32_t dstride, uint32_t w, uint32_t h, GkTiles tb,
                                                      int32_t shift, int vec) {
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
    auto put = [&](int k, int ly, int lx, int32_t r0, int32_t g0, int32_t b0) {
        if (NC == 3) {
            const float a_r = 0.299f, a_g = 0.587f, a_b = 0.114f;
            const float cb = 0.5f / (1.0f - a_b), cr = 0.5f / (1.0f - a_r);
            const float r = (float)(r0 - shift), g = (float)(g0 - shift), b = (float)(b0 - shift);
            const float t0 = a_r * r, t1 = a_g * g, t2 = a_b * b;
            const float Y = (t0 + t1) + t2;
            T[ly][lx] = Y;
            U[k] = cb * (b - Y);
            V[k] = cr * (r - Y);
        } else {
            T[ly][lx] = (float)(r0 - shift);
        }
    };
    const bool inner = fullw97(x0, (int)w);
    if (inner) {
        // (x0 is a multiple of 128, so every main group is aligned when the plane rows are; a
        // halo group outside the resolution is read one mirrored sample at a time)
        const bool v = vec && al4(p0) && al4(p1) && al4(p2);
        fwd97_groups(tid, [&](int g, int ly, int lx) {
            const size_t r = (size_t)mirror97(y0 - T97_HALO + ly, (int)h) * sin;
            const int gx = x0 - T97_HALO + lx;
            int4 a, b, c;
            if (gx >= 0 && gx + 3 < (int)w) {
                const size_t i = r + gx;
                a = ld4v(p0 + i, v);
                b = NC == 3 ? ld4v(p1 + i, v) : a; c = NC == 3 ? ld4v(p2 + i, v) : a;
            } else {
                int ga[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) ga[j] = mirror97(gx + j, (int)w);
                a = make_int4((int32_t)p0[r + ga[0]], (int32_t)p0[r + ga[1]], (int32_t)p0[r + ga[2]], (int32_t)p0[r + ga[3]]);
                b = NC == 3 ? make_int4((int32_t)p1[r + ga[0]], (int32_t)p1[r + ga[1]], (int32_t)p1[r + ga[2]], (int32_t)p1[r + ga[3]]) : a;
                c = NC == 3 ? make_int4((int32_t)p2[r + ga[0]], (int32_t)p2[r + ga[1]], (int32_t)p2[r + ga[2]], (int32_t)p2[r + ga[3]]) : a;
            }
            put(4 * g, ly, lx, a.x, b.x, c.x);
            put(4 * g + 1, ly, lx + 1, a.y, b.y, c.y);
            put(4 * g + 2, ly, lx + 2, a.z, b.z, c.z);
            put(4 * g + 3, ly, lx + 3, a.w, b.w, c.w);
        });
    } else {
        fwd97_fill_slots(x0, y0, (int)w, (int)h, tid, [&](int k, int ly, int lx, int gy, int gx) {
            const size_t i = (size_t)gy * sin + gx;
            put(k, ly, lx, (int32_t)p0[i], (int32_t)p1[i], (int32_t)p2[i]);
        });
    }
    __syncthreads();
    fwd97_lift(T, (int)w, (int)h, tid);
    fwd97_store(T, dst, dstride, x0, y0, (int)w, (int)h, tid);
    if (NC == 3) {
#pragma unroll
        for (int c = 1; c < 3; ++c) {
            __syncthreads();
            if (inner) {
                fwd97_groups(tid, [&](int g, int ly, int lx) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) T[ly][lx + j] = c == 1 ? U[4 * g + j] : V[4 * g + j];
                });
            } else {
                fwd97_fill_slots(x0, y0, (int)w, (int)h, tid,
                                 [&](int k, int ly, int lx, int, int) { T[ly][lx] = c == 1 ? U[k] : V[k]; });
            }
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
// f(ly, lx, sy, sx, fac): interleaved position (ly, lx) from Mallat position (sy, sx), times the
// horizontal scaling of its column (2/K odd, K even; 1 when there is no horizontal pass)
template <class F>
__device__ __forceinline__ void inv97_fill(int x0, int y0, int w, int h, int tid, F f) {
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    const float fe = w > 1 ? F97_K : 1.0f, fo = w > 1 ? I97_TWO_INVK : 1.0f;
    if (fullw97(x0, w)) {   // (rows and halo columns mirrored)
        // even interleaved columns (lx even) are L samples x0/2 - 2 + lx/2, odd ones H samples
        const int tx = tid & 63, ty = tid >> 6, hx = x0 >> 1;
        for (int ly = ty; ly < T97_LH; ly += 4) {
            const int gy = mirror97(y0 - T97_HALO + ly, h), sy = (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1);
            f(ly, T97_HALO + 2 * tx, sy, hx + tx, fe);
            f(ly, T97_HALO + 1 + 2 * tx, sy, snw + hx + tx, fo);
        }
        for (int i = tid; i < 8 * T97_LH; i += 256) {
            const int ly = i >> 3, j = i & 7, lx = j < 4 ? j : 128 + j;
            const int gy = mirror97(y0 - T97_HALO + ly, h), sy = (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1);
            const int gx = mirror97(x0 - T97_HALO + lx, w);
            f(ly, lx, sy, (gx & 1) ? snw + (gx >> 1) : (gx >> 1), (lx & 1) ? fo : fe);
        }
    } else {
        for (int i = tid; i < T97_LH * T97_LW; i += 256) {
            const int ly = i / T97_LW, lx = i % T97_LW;
            const int gy = mirror97(y0 - T97_HALO + ly, h), gx = mirror97(x0 - T97_HALO + lx, w);
            f(ly, lx, (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1), (gx & 1) ? (snw + (gx >> 1)) : (gx >> 1), (lx & 1) ? fo : fe);
        }
    }
}

// k_dwt97_inv_l1's tile: rows of 140 floats (a multiple of four), so output column c (LDS
// column c + 4) of a 4-column group sits on a 16-byte boundary: one ds_read_b128 per group
typedef float Lds97i[T97_LH][T97_LW + 4];
template <class TT>
__device__ __forceinline__ void inv97_lift(TT& T, int w, int h, int tid) {
    const int tx = tid & 63, ty = tid >> 6;
    if (w > 1) {
        // step s (delta, gamma, beta, alpha) updates columns 2 + s, 4 + s, ... (67 - s) of every row
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float c = s == 0 ? I97_D : (s == 1 ? I97_G : (s == 2 ? I97_B : I97_A));
            const int first = 2 + s, e = 3 - s;
            auto upd = [&](int ly, int lx) {
                const float t = (T[ly][lx - 1] + T[ly][lx + 1]) * c;
                T[ly][lx] = T[ly][lx] + t;
            };
            for (int ly = ty; ly < T97_LH; ly += 4) upd(ly, first + 2 * tx);
            if (e && tid < T97_LH * e) upd(tid / e, first + 2 * (64 + tid % e));
            __syncthreads();
        }
    }
    if (h > 1) {
        // step s updates rows 2 + s, 4 + s, ... (19 - s rows) of the output columns 4..131; the
        // vertical scaling (2/K odd, K even rows) of every value steps 0 and 1 read is applied as
        // it is read, until that step has written it
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float c = s == 0 ? I97_D : (s == 1 ? I97_G : (s == 2 ? I97_B : I97_A));
            const int first = 2 + s, nrows = 19 - s;
            auto upd = [&](int ly, int lx) {
                if (s == 0) {   // even row, odd neighbours: nothing scaled yet
                    const float t = (T[ly - 1][lx] * I97_TWO_INVK + T[ly + 1][lx] * I97_TWO_INVK) * c;
                    T[ly][lx] = T[ly][lx] * F97_K + t;
                } else if (s == 1) {   // odd row; its even neighbours were written by step 0
                    const float t = (T[ly - 1][lx] + T[ly + 1][lx]) * c;
                    T[ly][lx] = T[ly][lx] * I97_TWO_INVK + t;
                } else {
                    const float t = (T[ly - 1][lx] + T[ly + 1][lx]) * c;
                    T[ly][lx] = T[ly][lx] + t;
                }
            };
            for (int m = ty; m < nrows; m += 4) {
                upd(first + 2 * m, T97_HALO + tx);
                upd(first + 2 * m, T97_HALO + 64 + tx);
            }
            __syncthreads();
        }
    }
}

// One level, cpw components per workgroup with the next one's input prefetched (as
// k_dwt97_fwd_level; the positions and scalings of inv97_fill's full-width path)
__global__ __launch_bounds__(256) void k_dwt97_inv_level(const float* __restrict__ src, uint32_t sstride,
                                                         float* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h, GkTiles tb, GkComps cs, uint32_t cpw) {
    __shared__ Lds97 T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z % tb.count(), c0 = bi.z / tb.count() * cpw, c1 = min(cs.n, c0 + cpw);
    src += tb.offset(tile, sstride);
    dst += tb.offset(tile, dstride);
    const int x0 = bi.x * T97_W, y0 = bi.y * T97_H, tid = threadIdx.x;
    const int tx = tid & 63, ty = tid >> 6, hx = x0 >> 1;
    constexpr int PF_ROWS = (T97_LH + 3) / 4, PF_HALO = (8 * T97_LH + 255) / 256;
    float PF[2 * PF_ROWS + PF_HALO];
    const bool inner = fullw97(x0, (int)w);
    const int snw = ((int)w + 1) >> 1, snh = ((int)h + 1) >> 1;
    const float fe = w > 1 ? F97_K : 1.0f, fo = w > 1 ? I97_TWO_INVK : 1.0f;
    auto srow = [&](int ly) {
        const int gy = mirror97(y0 - T97_HALO + ly, (int)h);
        return (size_t)((gy & 1) ? (snh + (gy >> 1)) : (gy >> 1)) * sstride;
    };
    auto hlx = [](int i) { const int j = i & 7; return j < 4 ? j : 128 + j; };
    auto fetch = [&](const float* sc) {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < T97_LH) {
                const float* r = sc + srow(ly) + hx + tx;
                PF[2 * m] = r[0];
                PF[2 * m + 1] = r[snw];
            }
        }
#pragma unroll
        for (int k = 0; k < PF_HALO; ++k) {
            const int i = tid + 256 * k;
            if (i < 8 * T97_LH) {
                const int gx = mirror97(x0 - T97_HALO + hlx(i), (int)w);
                PF[2 * PF_ROWS + k] = sc[srow(i >> 3) + ((gx & 1) ? snw + (gx >> 1) : (gx >> 1))];
            }
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < T97_LH) {
                T[ly][T97_HALO + 2 * tx] = PF[2 * m] * fe;
                T[ly][T97_HALO + 1 + 2 * tx] = PF[2 * m + 1] * fo;
            }
        }
#pragma unroll
        for (int k = 0; k < PF_HALO; ++k) {
            const int i = tid + 256 * k;
            if (i < 8 * T97_LH) T[i >> 3][hlx(i)] = PF[2 * PF_ROWS + k] * ((hlx(i) & 1) ? fo : fe);
        }
    };
    if (inner) fetch(src + c0 * cs.cstride);
    for (uint32_t c = c0; c < c1; ++c) {
        if (c != c0) __syncthreads();   // the previous component's stores have read the tile
        const float* sc = src + c * cs.cstride;
        if (inner) put();
        else inv97_fill(x0, y0, (int)w, (int)h, tid,
                        [&](int ly, int lx, int sy, int sx, float f) { T[ly][lx] = sc[(size_t)sy * sstride + sx] * f; });
        __syncthreads();
        if (inner && c + 1 < c1) fetch(sc + cs.cstride);
        inv97_lift(T, (int)w, (int)h, tid);
        float* dc = dst + c * cs.cstride;
        for (int ry = ty; ry < T97_H; ry += 4) {
            const int gy = y0 + ry;
            if (gy >= (int)h) break;
            float* drow = dc + (size_t)gy * dstride + x0;
            if (x0 + tx < (int)w) drow[tx] = T[ry + T97_HALO][T97_HALO + tx];
            if (x0 + 64 + tx < (int)w) drow[64 + tx] = T[ry + T97_HALO][T97_HALO + 64 + tx];
        }
    }
}

// Last inverse level into the caller's planes: inverse ICT for NC = 3 (mct.cpp:284-364,
// lrintf rounding), DC shift and clamp, only inside the output window (GkWin).  One LDS
// tile; the Y and U results of each thread's 16 output samples wait in registers.  A thread
// owns four groups of four consecutive columns (row i >> 5, columns 4 (i & 31) .. + 3 of
// group i = tid + 256 j), written as one vector store per plane where the window and the
// planes allow.
template <class TO, int NC>
__global__ __launch_bounds__(256) void k_dwt97_inv_l1(const float* __restrict__ src, uint64_t cstride, uint32_t sstride,
                                                      GkPtr3 out, uint32_t ostride, GkWin win, uint32_t w, uint32_t h,
                                                      GkTiles tb, int32_t shift, int32_t mn, int32_t mx, int vec) {
    __shared__ __attribute__((aligned(16))) Lds97i T;
    const uint3 bi = xcd_tile();
    const uint32_t tile = bi.z;
    src += tb.offset(tile, sstride);
    int32_t ox, oy;
    tb.origin(tile, ox, oy);
    const int x0 = bi.x * T97_W, y0 = bi.y * T97_H, tid = threadIdx.x;
    float R0[16], R1[16];
    // Full-width tiles: the next component's input is loaded into registers (PF, the positions
    // inv97_fill's full-width path visits) while the current one lifts (as k_dwt53_inv_l1).
    constexpr int PF_ROWS = (T97_LH + 3) / 4, PF_HALO = (8 * T97_LH + 255) / 256;
    float PF[2 * PF_ROWS + PF_HALO];
    const bool inner = fullw97(x0, (int)w);
    const int tx = tid & 63, ty = tid >> 6, hx = x0 >> 1;
    const int snw = ((int)w + 1) >> 1, snh = ((int)h + 1) >> 1;
    const float fe = w > 1 ? F97_K : 1.0f, fo = w > 1 ? I97_TWO_INVK : 1.0f;
    auto srow = [&](int ly) {
        const int gy = mirror97(y0 - T97_HALO + ly, (int)h);
        return (size_t)((gy & 1) ? (snh + (gy >> 1)) : (gy >> 1)) * sstride;
    };
    auto hlx = [](int i) { const int j = i & 7; return j < 4 ? j : 128 + j; };
    auto fetch = [&](const float* sc) {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < T97_LH) {
                const float* r = sc + srow(ly) + hx + tx;
                PF[2 * m] = r[0];
                PF[2 * m + 1] = r[snw];
            }
        }
#pragma unroll
        for (int k = 0; k < PF_HALO; ++k) {
            const int i = tid + 256 * k;
            if (i < 8 * T97_LH) {
                const int gx = mirror97(x0 - T97_HALO + hlx(i), (int)w);
                PF[2 * PF_ROWS + k] = sc[srow(i >> 3) + ((gx & 1) ? snw + (gx >> 1) : (gx >> 1))];
            }
        }
    };
    auto put = [&]() {
#pragma unroll
        for (int m = 0; m < PF_ROWS; ++m) {
            const int ly = ty + 4 * m;
            if (ly < T97_LH) {
                T[ly][T97_HALO + 2 * tx] = PF[2 * m] * fe;
                T[ly][T97_HALO + 1 + 2 * tx] = PF[2 * m + 1] * fo;
            }
        }
#pragma unroll
        for (int k = 0; k < PF_HALO; ++k) {
            const int i = tid + 256 * k;
            if (i < 8 * T97_LH) T[i >> 3][hlx(i)] = PF[2 * PF_ROWS + k] * ((hlx(i) & 1) ? fo : fe);
        }
    };
    if (inner) fetch(src);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (c) __syncthreads();
        const float* sc = src + c * cstride;
        if (inner) put();
        else inv97_fill(x0, y0, (int)w, (int)h, tid,
                        [&](int ly, int lx, int sy, int sx, float f) { T[ly][lx] = sc[(size_t)sy * sstride + sx] * f; });
        __syncthreads();
        if (inner && c + 1 < NC) fetch(sc + cstride);
        inv97_lift(T, (int)w, (int)h, tid);
        if (c + 1 < NC) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = tid + 256 * j;
                const float4 v = *(const float4*)&T[(i >> 5) + T97_HALO][4 * (i & 31) + T97_HALO];
                float* R = c == 0 ? R0 : R1;
                R[4 * j] = v.x; R[4 * j + 1] = v.y; R[4 * j + 2] = v.z; R[4 * j + 3] = v.w;
            }
        }
    }
    TO* o0 = (TO*)out.p[0];
    TO* o1 = (TO*)out.p[NC == 3 ? 1 : 0];
    TO* o2 = (TO*)out.p[NC == 3 ? 2 : 0];
    auto cl = [&](float f) { int32_t v = (int32_t)rintf(f) + shift; return v < mn ? mn : (v > mx ? mx : v); };
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = tid + 256 * j, ry = i >> 5, rx = 4 * (i & 31);
        const int gy = y0 + ry, gx = x0 + rx, X = ox + gx, Y = oy + gy;
        if (gy >= (int)h || Y < win.y0 || Y >= win.y1) continue;
        int32_t r[4], g[4], b[4];
        const float4 lv = *(const float4*)&T[ry + T97_HALO][rx + T97_HALO];
        const float lastv[4] = {lv.x, lv.y, lv.z, lv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float last = lastv[e];
            if (NC == 3) {
                const float Yv = R0[4 * j + e], U = R1[4 * j + e], V = last;
                const float R = Yv + 1.402f * V;
                const float G = (Yv - 0.34413f * U) - 0.71414f * V;
                const float B = Yv + 1.772f * U;
                r[e] = cl(R); g[e] = cl(G); b[e] = cl(B);
            } else {
                r[e] = cl(last);
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
    const uint32_t gx = (w + T97_W - 1) / T97_W, gy = (h + T97_H - 1) / T97_H;
    const uint32_t cpw = gk_dwt_cpw(gx * gy * tb.count(), cs.n, true);   // (gk_kernels.hip)
    const uint32_t ng = cpw > 1 ? cs.n : comps_in_grid97(tb, cs);
    for (uint32_t c = 0; c < cs.n; c += ng) {
        GkComps g = cs; g.n = ng;
        dim3 grid(gx, gy, tb.count() * (ng / cpw));
        hipLaunchKernelGGL(k_dwt97_fwd_level, grid, dim3(256), 0, st, src + c * cs.cstride, sstride, dst + c * cs.cstride,
                           dstride, w, h, tb, g, cpw);
    }
}
void gk_launch_dwt97_inv(hipStream_t st, const float* src, uint32_t sstride, float* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb, GkComps cs) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    const uint32_t gx = (w + T97_W - 1) / T97_W, gy = (h + T97_H - 1) / T97_H;
    const uint32_t cpw = gk_dwt_cpw(gx * gy * tb.count(), cs.n, false);   // (gk_kernels.hip)
    const uint32_t ng = cpw > 1 ? cs.n : comps_in_grid97(tb, cs);
    for (uint32_t c = 0; c < cs.n; c += ng) {
        GkComps g = cs; g.n = ng;
        dim3 grid(gx, gy, tb.count() * (ng / cpw));
        hipLaunchKernelGGL(k_dwt97_inv_level, grid, dim3(256), 0, st, src + c * cs.cstride, sstride, dst + c * cs.cstride,
                           dstride, w, h, tb, g, cpw);
    }
}
void gk_launch_dwt97_fwd_l1(hipStream_t st, int stype, int nc, GkPtr3 in, uint32_t sin, float* dst, uint64_t cstride,
                            uint32_t dstride, uint32_t w, uint32_t h, GkTiles tb, int32_t shift) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + T97_W - 1) / T97_W, (h + T97_H - 1) / T97_H, tb.count());
    const int vec = (sin & 3) == 0;   // (the kernel checks each tile's row pointers)
    if (nc == 3)
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt97_fwd_l1<T, 3>), grid, dim3(256), 0, st, in, sin, dst,
                                                        cstride, dstride, w, h, tb, shift, vec))
    else
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt97_fwd_l1<T, 1>), grid, dim3(256), 0, st, in, sin, dst,
                                                        cstride, dstride, w, h, tb, shift, vec))
}
void gk_launch_dwt97_inv_l1(hipStream_t st, int stype, int nc, const float* src, uint64_t cstride, uint32_t sstride,
                            GkPtr3 out, uint32_t ostride, GkWin win, uint32_t w, uint32_t h, GkTiles tb, int32_t shift,
                            int32_t mn, int32_t mx) {
    if (!w || !h || !tb.count()) return;   // an empty region (a resolution of zero width or height): no launch
    dim3 grid((w + T97_W - 1) / T97_W, (h + T97_H - 1) / T97_H, tb.count());
    const int vec = gk_vec_ok(gk_sample_size(stype), out, nc, ostride);
    if (nc == 3)
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt97_inv_l1<T, 3>), grid, dim3(256), 0, st, src, cstride,
                                                        sstride, out, ostride, win, w, h, tb, shift, mn, mx, vec))
    else
        GK_SAMPLE_DISPATCH(stype, T, hipLaunchKernelGGL((k_dwt97_inv_l1<T, 1>), grid, dim3(256), 0, st, src, cstride,
                                                        sstride, out, ostride, win, w, h, tb, shift, mn, mx, vec))
}
