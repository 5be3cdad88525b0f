// gk_kernels.hip — MI355X (gfx950) kernels for the JPEG 2000 tile pipeline.
//
// Stage map (reference → kernel), see DESIGN.md:
//   TileProcessor::dcLevelShiftCompress + mct CompressRev   → k_dc_rct_fwd / k_dc_fwd
//   dwt53::encode_and_deinterleave_v/h (WaveletFwd.cpp)      → k_dwt53_fwd_level
//   T1Part1::preCompress + T1::compress_cblk (T1.cpp)        → k_t1_encode
//   T1::decompress_cblk + ShiftFilter (T1.cpp, filters/)     → k_t1_decode
//   decompress_tile_53 (WaveletReverse.cpp)                  → k_dwt53_inv_level
//   mct DecompressRev + dcLevelShiftDecompress               → k_rct_inv_dc / k_dc_inv
//
// All kernels are wave64-native: block dims are multiples of 64, code-block
// kernels run one wave per code-block with lane = column.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"

#define LDS_BARRIER() __syncthreads()

// =============================================================================
// DC level shift + RCT (forward).  In: 3 planes (int32, stride sin), out: 3
// planes (stride sout).  mct.cpp:99-146, TileProcessor.cpp:506-535.
// =============================================================================
__global__ __launch_bounds__(256) void k_dc_rct_fwd(const int32_t* __restrict__ r_in, const int32_t* __restrict__ g_in,
                                                    const int32_t* __restrict__ b_in, uint32_t sin,
                                                    int32_t* __restrict__ y_out, int32_t* __restrict__ u_out,
                                                    int32_t* __restrict__ v_out, uint32_t sout, uint32_t w, uint32_t h,
                                                    int32_t shift) {
    uint32_t x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    uint32_t y = blockIdx.y;
    if (y >= h || x4 >= w) return;
    const int32_t* rp = r_in + (size_t)y * sin;
    const int32_t* gp = g_in + (size_t)y * sin;
    const int32_t* bp = b_in + (size_t)y * sin;
    int32_t* yp = y_out + (size_t)y * sout;
    int32_t* up = u_out + (size_t)y * sout;
    int32_t* vp = v_out + (size_t)y * sout;
    if (x4 + 3 < w && ((sin | sout) & 3) == 0) {
        int4 r = *(const int4*)(rp + x4), g = *(const int4*)(gp + x4), b = *(const int4*)(bp + x4);
        r.x -= shift; r.y -= shift; r.z -= shift; r.w -= shift;
        g.x -= shift; g.y -= shift; g.z -= shift; g.w -= shift;
        b.x -= shift; b.y -= shift; b.z -= shift; b.w -= shift;
        int4 Y, U, V;
        Y.x = (r.x + 2 * g.x + b.x) >> 2; Y.y = (r.y + 2 * g.y + b.y) >> 2;
        Y.z = (r.z + 2 * g.z + b.z) >> 2; Y.w = (r.w + 2 * g.w + b.w) >> 2;
        U.x = b.x - g.x; U.y = b.y - g.y; U.z = b.z - g.z; U.w = b.w - g.w;
        V.x = r.x - g.x; V.y = r.y - g.y; V.z = r.z - g.z; V.w = r.w - g.w;
        *(int4*)(yp + x4) = Y; *(int4*)(up + x4) = U; *(int4*)(vp + x4) = V;
    } else {
        for (uint32_t x = x4; x < w && x < x4 + 4; ++x) {
            int32_t r = rp[x] - shift, g = gp[x] - shift, b = bp[x] - shift;
            yp[x] = (r + 2 * g + b) >> 2; up[x] = b - g; vp[x] = r - g;
        }
    }
}

__global__ __launch_bounds__(256) void k_dc_fwd(const int32_t* __restrict__ in, uint32_t sin, int32_t* __restrict__ out,
                                                uint32_t sout, uint32_t w, uint32_t h, int32_t shift) {
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (y >= h || x >= w) return;
    out[(size_t)y * sout + x] = in[(size_t)y * sin + x] - shift;
}

// Inverse RCT + DC shift + clamp (mct.cpp:221-283).
__global__ __launch_bounds__(256) void k_rct_inv_dc(const int32_t* __restrict__ y_in, const int32_t* __restrict__ u_in,
                                                    const int32_t* __restrict__ v_in, uint32_t sin,
                                                    int32_t* __restrict__ r_out, int32_t* __restrict__ g_out,
                                                    int32_t* __restrict__ b_out, uint32_t sout, uint32_t w, uint32_t h,
                                                    int32_t shift, int32_t mn, int32_t mx) {
    uint32_t x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    uint32_t y = blockIdx.y;
    if (y >= h || x4 >= w) return;
    const int32_t* Yp = y_in + (size_t)y * sin;
    const int32_t* Up = u_in + (size_t)y * sin;
    const int32_t* Vp = v_in + (size_t)y * sin;
    int32_t* rp = r_out + (size_t)y * sout;
    int32_t* gp = g_out + (size_t)y * sout;
    int32_t* bp = b_out + (size_t)y * sout;
    auto cl = [&](int32_t v) { return v < mn ? mn : (v > mx ? mx : v); };
    if (x4 + 3 < w && ((sin | sout) & 3) == 0) {
        int4 Y = *(const int4*)(Yp + x4), U = *(const int4*)(Up + x4), V = *(const int4*)(Vp + x4);
        int4 R, G, B;
        G.x = Y.x - ((U.x + V.x) >> 2); G.y = Y.y - ((U.y + V.y) >> 2);
        G.z = Y.z - ((U.z + V.z) >> 2); G.w = Y.w - ((U.w + V.w) >> 2);
        R.x = cl(V.x + G.x + shift); R.y = cl(V.y + G.y + shift); R.z = cl(V.z + G.z + shift); R.w = cl(V.w + G.w + shift);
        B.x = cl(U.x + G.x + shift); B.y = cl(U.y + G.y + shift); B.z = cl(U.z + G.z + shift); B.w = cl(U.w + G.w + shift);
        G.x = cl(G.x + shift); G.y = cl(G.y + shift); G.z = cl(G.z + shift); G.w = cl(G.w + shift);
        *(int4*)(rp + x4) = R; *(int4*)(gp + x4) = G; *(int4*)(bp + x4) = B;
    } else {
        for (uint32_t x = x4; x < w && x < x4 + 4; ++x) {
            int32_t Y = Yp[x], U = Up[x], V = Vp[x];
            int32_t G = Y - ((U + V) >> 2);
            rp[x] = cl(V + G + shift); gp[x] = cl(G + shift); bp[x] = cl(U + G + shift);
        }
    }
}

__global__ __launch_bounds__(256) void k_dc_inv(const int32_t* __restrict__ in, uint32_t sin, int32_t* __restrict__ out,
                                                uint32_t sout, uint32_t w, uint32_t h, int32_t shift, int32_t mn,
                                                int32_t mx) {
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (y >= h || x >= w) return;
    int32_t v = in[(size_t)y * sin + x] + shift;
    out[(size_t)y * sout + x] = v < mn ? mn : (v > mx ? mx : v);
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
                                                         uint32_t h) {
    __shared__ int32_t T[DWT_LH][DWT_LW + 1];
    const int x0 = blockIdx.x * DWT_TW, y0 = blockIdx.y * DWT_TH;
    const int tid = threadIdx.x;
    // load rows y0-2 .. y0+TH, cols x0-2 .. x0+TW (mirrored)
    for (int i = tid; i < DWT_LH * DWT_LW; i += 256) {
        int ly = i / DWT_LW, lx = i % DWT_LW;
        int gy = mirror(y0 - 2 + ly, (int)h), gx = mirror(x0 - 2 + lx, (int)w);
        T[ly][lx] = src[(size_t)gy * sstride + gx];
    }
    LDS_BARRIER();
    if (h > 1) {
        // vertical predict: odd absolute rows y in [y0-1, y0+TH-1]  (local ly = y - y0 + 2, odd y <=> ly odd)
        for (int i = tid; i < (DWT_TH / 2 + 1) * DWT_LW; i += 256) {
            int k = i / DWT_LW, lx = i % DWT_LW;
            int ly = 1 + 2 * k;   // y = y0 - 1 + 2k
            T[ly][lx] -= (T[ly - 1][lx] + T[ly + 1][lx]) >> 1;
        }
        LDS_BARRIER();
        // vertical update: even rows y in [y0, y0+TH-2]: ly = 2 + 2k
        for (int i = tid; i < (DWT_TH / 2) * DWT_LW; i += 256) {
            int k = i / DWT_LW, lx = i % DWT_LW;
            int ly = 2 + 2 * k;
            T[ly][lx] += (T[ly - 1][lx] + T[ly + 1][lx] + 2) >> 2;
        }
        LDS_BARRIER();
    }
    if (w > 1) {
        // horizontal predict on rows ly in [2, TH+2): odd cols lx = 1 + 2k
        for (int i = tid; i < DWT_TH * (DWT_TW / 2 + 1); i += 256) {
            int ly = 2 + i / (DWT_TW / 2 + 1), k = i % (DWT_TW / 2 + 1);
            int lx = 1 + 2 * k;
            T[ly][lx] -= (T[ly][lx - 1] + T[ly][lx + 1]) >> 1;
        }
        LDS_BARRIER();
        for (int i = tid; i < DWT_TH * (DWT_TW / 2); i += 256) {
            int ly = 2 + i / (DWT_TW / 2), k = i % (DWT_TW / 2);
            int lx = 2 + 2 * k;
            T[ly][lx] += (T[ly][lx - 1] + T[ly][lx + 1] + 2) >> 2;
        }
        LDS_BARRIER();
    }
    // scatter to quadrants
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    for (int i = tid; i < DWT_TH * DWT_TW; i += 256) {
        int ry = i / DWT_TW, rx = i % DWT_TW;
        // iterate so that consecutive threads write consecutive outputs of one quadrant row:
        int q = rx / (DWT_TW / 2);           // 0: even columns (L), 1: odd columns (H)
        int k = rx % (DWT_TW / 2);
        int gx = x0 + 2 * k + q, gy = y0 + ry;
        if (gx >= (int)w || gy >= (int)h) continue;
        int32_t v = T[ry + 2][2 + 2 * k + q];
        int ox = (q == 0) ? (gx >> 1) : (snw + (gx >> 1));
        int oy = ((gy & 1) == 0) ? (gy >> 1) : (snh + (gy >> 1));
        dst[(size_t)oy * dstride + ox] = v;
    }
}

// Inverse 5/3 level (WaveletReverse.cpp:802-879): horizontal then vertical,
// on the interleaved signal with symmetric extension.  Output tile rows
// y0..y0+TH-1; needs interleaved rows y0-1..y0+TH+1 and cols x0-1..x0+TW+1.
#define IDWT_LW (DWT_TW + 3)
#define IDWT_LH (DWT_TH + 3)
__global__ __launch_bounds__(256) void k_dwt53_inv_level(const int32_t* __restrict__ src, uint32_t sstride,
                                                         int32_t* __restrict__ dst, uint32_t dstride, uint32_t w,
                                                         uint32_t h) {
    __shared__ int32_t T[IDWT_LH][IDWT_LW + 1];
    const int x0 = blockIdx.x * DWT_TW, y0 = blockIdx.y * DWT_TH;
    const int tid = threadIdx.x;
    const int snw = (w + 1) >> 1, snh = (h + 1) >> 1;
    for (int i = tid; i < IDWT_LH * IDWT_LW; i += 256) {
        int ly = i / IDWT_LW, lx = i % IDWT_LW;
        int gy = mirror(y0 - 1 + ly, (int)h), gx = mirror(x0 - 1 + lx, (int)w);
        int sy = (gy & 1) ? (snh + (gy >> 1)) : (gy >> 1);
        int sx = (gx & 1) ? (snw + (gx >> 1)) : (gx >> 1);
        T[ly][lx] = src[(size_t)sy * sstride + sx];
    }
    LDS_BARRIER();
    if (w > 1) {
        // horizontal step 1: even interleaved cols x (lx = x - x0 + 1): x even <=> lx odd, lx in [1, TW+1]
        for (int i = tid; i < IDWT_LH * (DWT_TW / 2 + 1); i += 256) {
            int ly = i / (DWT_TW / 2 + 1), k = i % (DWT_TW / 2 + 1);
            int lx = 1 + 2 * k;
            T[ly][lx] -= (T[ly][lx - 1] + T[ly][lx + 1] + 2) >> 2;
        }
        LDS_BARRIER();
        // step 2: odd cols x in [x0+1, x0+TW-1]: lx = 2 + 2k
        for (int i = tid; i < IDWT_LH * (DWT_TW / 2); i += 256) {
            int ly = i / (DWT_TW / 2), k = i % (DWT_TW / 2);
            int lx = 2 + 2 * k;
            T[ly][lx] += (T[ly][lx - 1] + T[ly][lx + 1]) >> 1;
        }
        LDS_BARRIER();
    }
    if (h > 1) {
        for (int i = tid; i < (DWT_TH / 2 + 1) * DWT_TW; i += 256) {
            int k = i / DWT_TW, lx = 1 + i % DWT_TW;
            int ly = 1 + 2 * k;
            T[ly][lx] -= (T[ly - 1][lx] + T[ly + 1][lx] + 2) >> 2;
        }
        LDS_BARRIER();
        for (int i = tid; i < (DWT_TH / 2) * DWT_TW; i += 256) {
            int k = i / DWT_TW, lx = 1 + i % DWT_TW;
            int ly = 2 + 2 * k;
            T[ly][lx] += (T[ly - 1][lx] + T[ly + 1][lx]) >> 1;
        }
        LDS_BARRIER();
    }
    for (int i = tid; i < DWT_TH * DWT_TW; i += 256) {
        int ry = i / DWT_TW, rx = i % DWT_TW;
        int gx = x0 + rx, gy = y0 + ry;
        if (gx >= (int)w || gy >= (int)h) continue;
        dst[(size_t)gy * dstride + gx] = T[ry + 1][rx + 1];
    }
}

#include "gk_t1_common.h"

// Shared per-wave T1 state.  Row bitmaps: bit x = column x; rows are stored
// with one guard row above and below (index y + 1).
struct T1Lds {
    uint64_t sig[66];
    uint64_t neg[66];
    uint64_t pi[64];
    uint64_t mu[64];
    uint64_t bit[64];
    uint32_t mq[47];
    uint8_t zc[512];
    uint8_t sc[256];
    uint8_t ctx[GK_CTX];    // state index | mps << 7
};

__device__ __forceinline__ void t1_init_tables(T1Lds& L, uint32_t orient) {
    const int lane = threadIdx.x;
    for (int i = lane; i < 512; i += 64) L.zc[i] = zc_rule(orient, (uint32_t)i);
    for (int i = lane; i < 256; i += 64) L.sc[i] = sc_rule((uint32_t)i);
    if (lane < 47) L.mq[lane] = c_mq[lane];
    if (lane < GK_CTX) L.ctx[lane] = (lane == CTX_UNI) ? 46 : (lane == CTX_AGG ? 3 : (lane == CTX_ZC ? 4 : 0));
}

// 3-bit window of a row around column x: bit0 = x-1, bit1 = x, bit2 = x+1
__device__ __forceinline__ uint32_t win3(uint64_t row, uint32_t x) {
    return (uint32_t)((x ? (row >> (x - 1)) : (row << 1)) & 7);
}
__device__ __forceinline__ uint32_t nbr9(uint64_t up, uint64_t mid, uint64_t dn, uint32_t x) {
    return win3(up, x) | ((win3(mid, x) & 5) << 3) | (win3(dn, x) << 6);
}
__device__ __forceinline__ uint32_t sc_index(uint64_t su, uint64_t nu, uint64_t sm, uint64_t nm, uint64_t sd,
                                             uint64_t nd, uint32_t x) {
    uint32_t wv = x ? (uint32_t)((sm >> (x - 1)) & 1) : 0, wn = x ? (uint32_t)((nm >> (x - 1)) & 1) : 0;
    uint32_t ev = (uint32_t)((sm >> (x + 1)) & 1) & (x < 63), en = (uint32_t)((nm >> (x + 1)) & 1) & (x < 63);
    uint32_t nv = (uint32_t)((su >> x) & 1), nn = (uint32_t)((nu >> x) & 1);
    uint32_t sv = (uint32_t)((sd >> x) & 1), sn = (uint32_t)((nd >> x) & 1);
    return (wn & wv) | (wv << 1) | ((en & ev) << 2) | (ev << 3) | ((nn & nv) << 4) | (nv << 5) | ((sn & sv) << 6) |
           (sv << 7);
}

// ---------------------------------------------------------------- MQ encoder
struct MqE {
    uint32_t a, c, ct;
    int32_t bp;        // index of current byte (-1 = pad byte before the buffer)
    uint32_t cur;      // value of byte at bp (not yet stored)
    uint8_t* out;      // block slot (out[-1] is the zero pad)
    uint32_t cap;
    int overflow;
};
__device__ __forceinline__ void mq_emit(MqE& m, uint32_t newbyte) {
    if (m.bp >= 0) {
        if ((uint32_t)m.bp < m.cap) m.out[m.bp] = (uint8_t)m.cur; else m.overflow = 1;
    }
    m.bp++;
    m.cur = newbyte & 0xff;
}
__device__ __forceinline__ void mq_byteout(MqE& m) {
    if (m.cur == 0xff) {
        mq_emit(m, m.c >> 20); m.c &= 0xfffff; m.ct = 7;
    } else if ((m.c & 0x8000000) == 0) {
        mq_emit(m, m.c >> 19); m.c &= 0x7ffff; m.ct = 8;
    } else {
        m.cur++;
        if (m.cur == 0xff) {
            m.c &= 0x7ffffff; mq_emit(m, m.c >> 20); m.c &= 0xfffff; m.ct = 7;
        } else {
            mq_emit(m, m.c >> 19); m.c &= 0x7ffff; m.ct = 8;
        }
    }
}
__device__ __forceinline__ void mq_encode(MqE& m, T1Lds& L, uint32_t cx, uint32_t d) {
    uint32_t s = L.ctx[cx];
    uint32_t st = s & 0x7f, mps = s >> 7;
    uint32_t e = L.mq[st];
    uint32_t qe = e & 0xffff;
    m.a -= qe;
    if (mps == d) {
        if ((m.a & 0x8000) == 0) {
            if (m.a < qe) m.a = qe; else m.c += qe;
            L.ctx[cx] = (uint8_t)(((e >> 16) & 0x3f) | (mps << 7));
        } else { m.c += qe; return; }
    } else {
        if (m.a < qe) m.c += qe; else m.a = qe;
        L.ctx[cx] = (uint8_t)(((e >> 22) & 0x3f) | ((mps ^ (e >> 28)) << 7));
    }
    do {
        m.a <<= 1; m.c <<= 1;
        if (--m.ct == 0) mq_byteout(m);
    } while ((m.a & 0x8000) == 0);
}
__device__ __forceinline__ void mq_flush(MqE& m) {
    uint32_t tempc = m.c + m.a;
    m.c |= 0xffff;
    if (m.c >= tempc) m.c -= 0x8000;
    m.c <<= m.ct; mq_byteout(m);
    m.c <<= m.ct; mq_byteout(m);
    if (m.cur != 0xff) mq_emit(m, 0);   // advance: current byte becomes final
}

// =============================================================================
// T1 encode: one wave per code-block.  Lanes hold the block's columns in VGPRs
// (magnitudes << 6 as in T1Part1::preCompress), build per-plane row bitmaps
// with 64-bit ballots, then lane 0 runs the three coding passes per bit-plane
// (T1.cpp:498-780) on the LDS row bitmaps and the MQ coder (mqc_enc.cpp).
// Pass bookkeeping (rates, termination, monotone fix, FF back-off) follows
// T1.cpp:781-932 exactly.
// =============================================================================
__global__ __launch_bounds__(64) void k_t1_encode(const int32_t* __restrict__ coef, GkBlock* __restrict__ blocks,
                                                  uint8_t* __restrict__ bytes, GkPass* __restrict__ passes,
                                                  uint32_t* __restrict__ info, uint32_t nblocks, int* err) {
    __shared__ T1Lds L;
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const int lane = threadIdx.x;
    const GkBlock B = blocks[b];
    const uint32_t w = B.w, h = B.h;
    t1_init_tables(L, B.orient);
    // ---- load column `lane` (quantise + SMR, T1Part1.cpp:36-87)
    uint32_t m[64];
    uint64_t negrow[64];
    const bool irrev = B.flags & 1;
    uint32_t mx = 0;
#pragma unroll
    for (int y = 0; y < 64; ++y) {
        int32_t v = 0;
        if (y < (int)h && lane < (int)w) {
            int32_t raw = coef[B.band_off + (size_t)y * B.stride + lane];
            if (irrev) {
                float f = (__int_as_float(raw) / B.step) * 64.0f;   // T1Part1.cpp:74-75
                v = (int32_t)rintf(f);
            } else v = raw * 64;
        }
        uint32_t a = (uint32_t)(v < 0 ? -v : v);
        m[y] = a;
        mx = a > mx ? a : mx;
        negrow[y] = __ballot(v < 0);
    }
    for (int off = 32; off > 0; off >>= 1) { uint32_t o = __shfl_xor(mx, off); mx = o > mx ? o : mx; }
    uint32_t numbps = 0;
    if (mx) {
        uint32_t t = 32 - __clz(mx);
        numbps = t <= 6 ? 0 : t - 6;
    }
    if (lane < 66) { L.sig[lane] = 0; L.neg[lane] = 0; }
    if (lane < 2) { L.sig[64 + lane] = 0; L.neg[64 + lane] = 0; }
    if (lane == 0) {
        for (int y = 0; y < 64; ++y) { L.pi[y] = 0; L.mu[y] = 0; }
    }
#pragma unroll
    for (int y = 0; y < 64; ++y) if (lane == 0) L.neg[y + 1] = negrow[y];
    LDS_BARRIER();
    uint8_t* out = bytes + B.data_off;
    GkPass* P = passes + (size_t)b * GK_MAX_PASSES;
    if (numbps == 0) {
        if (lane == 0) { info[3 * b] = 0; info[3 * b + 1] = 0; info[3 * b + 2] = 0; }
        return;
    }
    MqE q;
    q.a = 0x8000; q.c = 0; q.ct = 12; q.bp = -1; q.cur = 0; q.out = out; q.cap = B.data_cap; q.overflow = 0;
    int passno = 0;
    const uint64_t wmask = (w >= 64) ? ~0ull : ((1ull << w) - 1);
    for (int bpno = (int)numbps - 1; bpno >= 0; --bpno) {
        // plane bitmap via ballots
#pragma unroll
        for (int y = 0; y < 64; ++y) {
            uint64_t r = __ballot((m[y] >> (bpno + 6)) & 1);
            if (lane == 0 && y < (int)h) L.bit[y] = r;
        }
        LDS_BARRIER();
        if (lane == 0) {
            for (int pt = (bpno == (int)numbps - 1) ? 2 : 0; pt < 3; ++pt) {
                if (pt == 0) {
                    // ---- significance propagation (T1.cpp:498-549)
                    for (uint32_t k = 0; k < h; k += 4) {
                        uint32_t nr = h - k < 4 ? h - k : 4;
                        uint64_t S[6], N[6], PI[4], BT[4];
                        for (int r = 0; r < 6; ++r) { S[r] = L.sig[k + r]; N[r] = L.neg[k + r]; }
                        for (uint32_t r = 0; r < nr; ++r) { PI[r] = L.pi[k + r]; BT[r] = L.bit[k + r]; }
                        for (uint32_t r = nr; r < 4; ++r) { PI[r] = ~0ull; BT[r] = 0; }
                        for (uint32_t x = 0; x < w; ++x) {
                            for (uint32_t r = 0; r < nr; ++r) {
                                uint64_t bx = 1ull << x;
                                if ((S[r + 1] | PI[r]) & bx) continue;
                                uint32_t f = nbr9(S[r], S[r + 1], S[r + 2], x);
                                if (!f) continue;
                                uint32_t v = (BT[r] >> x) & 1;
                                mq_encode(q, L, CTX_ZC + L.zc[f], v);
                                if (v) {
                                    uint32_t si = sc_index(S[r], N[r], S[r + 1], N[r + 1], S[r + 2], N[r + 2], x);
                                    uint32_t e = L.sc[si];
                                    uint32_t sg = (uint32_t)((L.neg[k + r + 1] >> x) & 1);
                                    mq_encode(q, L, CTX_SC + (e & 15), sg ^ (e >> 4));
                                    S[r + 1] |= bx;
                                    if (sg) N[r + 1] |= bx;
                                }
                                PI[r] |= bx;
                            }
                        }
                        for (uint32_t r = 0; r < nr; ++r) { L.sig[k + r + 1] = S[r + 1]; L.neg[k + r + 1] = N[r + 1]; L.pi[k + r] = PI[r]; }
                    }
                } else if (pt == 1) {
                    // ---- magnitude refinement (T1.cpp:572-623)
                    for (uint32_t k = 0; k < h; k += 4) {
                        uint32_t nr = h - k < 4 ? h - k : 4;
                        uint64_t S[6];
                        for (int r = 0; r < 6; ++r) S[r] = L.sig[k + r];
                        for (uint32_t x = 0; x < w; ++x) {
                            for (uint32_t r = 0; r < nr; ++r) {
                                uint64_t bx = 1ull << x;
                                uint64_t pir = L.pi[k + r];
                                if (!(S[r + 1] & bx) || (pir & bx)) continue;
                                uint64_t mur = L.mu[k + r];
                                uint32_t cx;
                                if (mur & bx) cx = CTX_MAG + 2;
                                else cx = nbr9(S[r], S[r + 1], S[r + 2], x) ? CTX_MAG + 1 : CTX_MAG;
                                mq_encode(q, L, cx, (uint32_t)((L.bit[k + r] >> x) & 1));
                                L.mu[k + r] = mur | bx;
                            }
                        }
                    }
                } else {
                    // ---- cleanup (T1.cpp:624-780)
                    for (uint32_t k = 0; k < h; k += 4) {
                        uint32_t nr = h - k < 4 ? h - k : 4;
                        uint64_t S[6], N[6], PI[4], BT[4];
                        for (int r = 0; r < 6; ++r) { S[r] = L.sig[k + r]; N[r] = L.neg[k + r]; }
                        for (uint32_t r = 0; r < 4; ++r) { PI[r] = r < nr ? L.pi[k + r] : 0; BT[r] = r < nr ? L.bit[k + r] : 0; }
                        for (uint32_t x = 0; x < w; ++x) {
                            uint64_t bx = 1ull << x;
                            uint32_t r = 0;
                            bool partial = false;
                            if (nr == 4) {
                                // aggregation: all four insignificant, unvisited, zero context
                                bool agg = true;
                                for (uint32_t rr = 0; rr < 4 && agg; ++rr) {
                                    if ((S[rr + 1] | PI[rr]) & bx) agg = false;
                                    else if (nbr9(S[rr], S[rr + 1], S[rr + 2], x)) agg = false;
                                }
                                if (agg && !((L.mu[k] | L.mu[k + 1] | L.mu[k + 2] | L.mu[k + 3]) & bx)) {
                                    uint32_t runlen = 0;
                                    for (; runlen < 4; ++runlen) if ((BT[runlen] >> x) & 1) break;
                                    mq_encode(q, L, CTX_AGG, runlen != 4);
                                    if (runlen == 4) continue;
                                    mq_encode(q, L, CTX_UNI, runlen >> 1);
                                    mq_encode(q, L, CTX_UNI, runlen & 1);
                                    r = runlen;
                                    partial = true;
                                }
                            }
                            for (; r < nr; ++r) {
                                if (!partial) {
                                    if ((S[r + 1] | PI[r]) & bx) continue;
                                    uint32_t f = nbr9(S[r], S[r + 1], S[r + 2], x);
                                    uint32_t v = (BT[r] >> x) & 1;
                                    mq_encode(q, L, CTX_ZC + L.zc[f], v);
                                    if (!v) continue;
                                }
                                partial = false;
                                uint32_t si = sc_index(S[r], N[r], S[r + 1], N[r + 1], S[r + 2], N[r + 2], x);
                                uint32_t e = L.sc[si];
                                uint32_t sg = (uint32_t)((L.neg[k + r + 1] >> x) & 1);
                                mq_encode(q, L, CTX_SC + (e & 15), sg ^ (e >> 4));
                                S[r + 1] |= bx;
                                if (sg) N[r + 1] |= bx;
                            }
                        }
                        for (uint32_t r = 0; r < nr; ++r) { L.sig[k + r + 1] = S[r + 1]; L.neg[k + r + 1] = N[r + 1]; L.pi[k + r] = 0; }
                    }
                }
                // ---- pass bookkeeping (T1.cpp:856-897)
                GkPass& ps = P[passno];
                if (pt == 2 && bpno == 0) {
                    mq_flush(q);
                    ps.term = 1; ps.rate = (uint32_t)q.bp;
                } else {
                    uint32_t extra = 5 + (q.ct < 5 ? 1 : 0);
                    ps.term = 0; ps.rate = (uint32_t)q.bp + extra;
                }
                ps.dist = 0.f;
                ++passno;
            }
        }
        LDS_BARRIER();
    }
    if (lane == 0) {
        // store the trailing byte if the flush left it pending (it is part of the stream
        // only when it precedes bp; numbytes = bp)
        uint32_t nbytes = (uint32_t)q.bp;
        if (q.bp >= 0 && (uint32_t)q.bp < q.cap) out[q.bp] = (uint8_t)q.cur;
        __threadfence_block();
        uint32_t last = nbytes;
        for (int i = passno; i > 0;) {                 // monotone rates (T1.cpp:907-919)
            GkPass& ps = P[--i];
            if (ps.rate > last) ps.rate = last; else last = ps.rate;
        }
        uint32_t prev = 0;
        for (int i = 0; i < passno; ++i) {             // FF back-off (T1.cpp:920-930)
            GkPass& ps = P[i];
            if (ps.rate > 0 && out[ps.rate - 1] == 0xff) ps.rate--;
            ps.len = ps.rate - prev;
            prev = ps.rate;
        }
        info[3 * b] = numbps;
        info[3 * b + 1] = (uint32_t)passno;
        info[3 * b + 2] = passno ? P[passno - 1].rate : 0;
        if (q.overflow) atomicOr(err, 1);
    }
}

// ---------------------------------------------------------------- MQ decoder
struct MqD {
    const uint8_t* buf;
    uint32_t len, bp;
    uint32_t a, c, ct;
};
__device__ __forceinline__ uint32_t mqd_at(const MqD& m, uint32_t i) { return i < m.len ? m.buf[i] : 0xffu; }
__device__ __forceinline__ void mqd_bytein(MqD& m) {
    uint32_t cur = mqd_at(m, m.bp), nxt = mqd_at(m, m.bp + 1);
    if (cur == 0xff) {
        if (nxt > 0x8f) { m.c += 0xff00; m.ct = 8; }
        else { m.bp++; m.c += nxt << 9; m.ct = 7; }
    } else { m.bp++; m.c += nxt << 8; m.ct = 8; }
}
__device__ __forceinline__ uint32_t mq_decode(MqD& m, T1Lds& L, uint32_t cx) {
    uint32_t s = L.ctx[cx];
    uint32_t st = s & 0x7f, mps = s >> 7;
    uint32_t e = L.mq[st];
    uint32_t qe = e & 0xffff;
    uint32_t d;
    m.a -= qe;
    if (m.c < (qe << 16)) {
        if (m.a < qe) { d = mps; L.ctx[cx] = (uint8_t)(((e >> 16) & 0x3f) | (mps << 7)); }
        else { d = mps ^ 1; L.ctx[cx] = (uint8_t)(((e >> 22) & 0x3f) | ((mps ^ (e >> 28)) << 7)); }
        m.a = qe;
    } else {
        m.c -= qe << 16;
        if ((m.a & 0x8000) != 0) return mps;
        if (m.a < qe) { d = mps ^ 1; L.ctx[cx] = (uint8_t)(((e >> 22) & 0x3f) | ((mps ^ (e >> 28)) << 7)); }
        else { d = mps; L.ctx[cx] = (uint8_t)(((e >> 16) & 0x3f) | (mps << 7)); }
    }
    do {
        if (m.ct == 0) mqd_bytein(m);
        m.a <<= 1; m.c <<= 1; m.ct--;
    } while ((m.a & 0x8000) == 0);
    return d;
}

// =============================================================================
// T1 decode: one wave per code-block (T1.cpp:934-1446).  Lane 0 decodes the
// passes on LDS row bitmaps; after each bit-plane the wave folds the plane's
// decoded bits into per-lane column magnitudes (lane = column, 64 VGPRs).
// Output is written after dequantisation (ShiftFilter v/2 or ScaleFilter
// v*step/2, filters/PostDecompressFilters.h) straight into the band window.
// =============================================================================
__global__ __launch_bounds__(64) void k_t1_decode(const uint8_t* __restrict__ bytes, const GkBlock* __restrict__ blocks,
                                                  int32_t* __restrict__ coef, uint32_t nblocks) {
    __shared__ T1Lds L;
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const int lane = threadIdx.x;
    const GkBlock B = blocks[b];
    const uint32_t w = B.w, h = B.h;
    t1_init_tables(L, B.orient);
    if (lane < 66) { L.sig[lane] = 0; L.neg[lane] = 0; }
    if (lane < 2) { L.sig[64 + lane] = 0; L.neg[64 + lane] = 0; }
    if (lane == 0) for (int y = 0; y < 64; ++y) { L.pi[y] = 0; L.mu[y] = 0; L.bit[y] = 0; }
    LDS_BARRIER();
    uint32_t M[64];
#pragma unroll
    for (int y = 0; y < 64; ++y) M[y] = 0;
    uint32_t npasses = B.npasses, numbps = B.numbps;
    MqD q;
    q.buf = bytes + B.data_off; q.len = B.len; q.bp = 0;
    // INITDEC (mqc_dec.cpp:98-112)
    q.c = (uint32_t)((B.len == 0 ? 0xffu : mqd_at(q, 0)) << 16);
    mqd_bytein(q);
    q.c <<= 7; q.ct -= 7; q.a = 0x8000;
    int bpno1 = (int)numbps;
    int passtype = 2;
    uint32_t p = 0;
    int lastplane = 0;          // bpno1 of the last plane folded
    bool partial_last = false;  // last plane ended before its cleanup pass
    uint64_t stale = 0;         // rows (bit y) significant before the final partial plane but not refined in it
    while (p < npasses && bpno1 >= 1) {
        // decode up to three passes of this plane
        int first_pt = passtype;
        int pt_done = 0;
        if (lane == 0) {
            for (int pt = first_pt; pt < 3 && p < npasses; ++pt, ++p, ++pt_done) {
                if (pt == 0) {
                    for (uint32_t k = 0; k < h; k += 4) {
                        uint32_t nr = h - k < 4 ? h - k : 4;
                        uint64_t S[6], N[6], PI[4], BT[4];
                        for (int r = 0; r < 6; ++r) { S[r] = L.sig[k + r]; N[r] = L.neg[k + r]; }
                        for (uint32_t r = 0; r < nr; ++r) { PI[r] = L.pi[k + r]; BT[r] = L.bit[k + r]; }
                        for (uint32_t r = nr; r < 4; ++r) { PI[r] = ~0ull; BT[r] = 0; }
                        for (uint32_t x = 0; x < w; ++x) {
                            for (uint32_t r = 0; r < nr; ++r) {
                                uint64_t bx = 1ull << x;
                                if ((S[r + 1] | PI[r]) & bx) continue;
                                uint32_t f = nbr9(S[r], S[r + 1], S[r + 2], x);
                                if (!f) continue;
                                if (mq_decode(q, L, CTX_ZC + L.zc[f])) {
                                    uint32_t si = sc_index(S[r], N[r], S[r + 1], N[r + 1], S[r + 2], N[r + 2], x);
                                    uint32_t e = L.sc[si];
                                    uint32_t sg = mq_decode(q, L, CTX_SC + (e & 15)) ^ (e >> 4);
                                    S[r + 1] |= bx;
                                    if (sg) N[r + 1] |= bx;
                                    BT[r] |= bx;
                                }
                                PI[r] |= bx;
                            }
                        }
                        for (uint32_t r = 0; r < nr; ++r) {
                            L.sig[k + r + 1] = S[r + 1]; L.neg[k + r + 1] = N[r + 1]; L.pi[k + r] = PI[r]; L.bit[k + r] = BT[r];
                        }
                    }
                } else if (pt == 1) {
                    for (uint32_t k = 0; k < h; k += 4) {
                        uint32_t nr = h - k < 4 ? h - k : 4;
                        uint64_t S[6];
                        for (int r = 0; r < 6; ++r) S[r] = L.sig[k + r];
                        for (uint32_t x = 0; x < w; ++x) {
                            for (uint32_t r = 0; r < nr; ++r) {
                                uint64_t bx = 1ull << x;
                                uint64_t pir = L.pi[k + r];
                                if (!(S[r + 1] & bx) || (pir & bx)) continue;
                                uint64_t mur = L.mu[k + r];
                                uint32_t cx;
                                if (mur & bx) cx = CTX_MAG + 2;
                                else cx = nbr9(S[r], S[r + 1], S[r + 2], x) ? CTX_MAG + 1 : CTX_MAG;
                                if (mq_decode(q, L, cx)) L.bit[k + r] |= bx;
                                L.mu[k + r] = mur | bx;
                                L.pi[k + r] = pir | bx;   // mark "coded in this plane" for the fold
                            }
                        }
                    }
                } else {
                    for (uint32_t k = 0; k < h; k += 4) {
                        uint32_t nr = h - k < 4 ? h - k : 4;
                        uint64_t S[6], N[6], PI[4], BT[4];
                        for (int r = 0; r < 6; ++r) { S[r] = L.sig[k + r]; N[r] = L.neg[k + r]; }
                        for (uint32_t r = 0; r < 4; ++r) { PI[r] = r < nr ? L.pi[k + r] : 0; BT[r] = r < nr ? L.bit[k + r] : 0; }
                        for (uint32_t x = 0; x < w; ++x) {
                            uint64_t bx = 1ull << x;
                            uint32_t r = 0;
                            bool partial = false;
                            if (nr == 4) {
                                bool agg = true;
                                for (uint32_t rr = 0; rr < 4 && agg; ++rr) {
                                    if ((S[rr + 1] | PI[rr]) & bx) agg = false;
                                    else if (nbr9(S[rr], S[rr + 1], S[rr + 2], x)) agg = false;
                                }
                                if (agg && !((L.mu[k] | L.mu[k + 1] | L.mu[k + 2] | L.mu[k + 3]) & bx)) {
                                    if (!mq_decode(q, L, CTX_AGG)) continue;
                                    uint32_t rl = mq_decode(q, L, CTX_UNI);
                                    rl = (rl << 1) | mq_decode(q, L, CTX_UNI);
                                    r = rl;
                                    partial = true;
                                }
                            }
                            for (; r < nr; ++r) {
                                if (!partial) {
                                    if ((S[r + 1] | PI[r]) & bx) continue;
                                    uint32_t f = nbr9(S[r], S[r + 1], S[r + 2], x);
                                    if (!mq_decode(q, L, CTX_ZC + L.zc[f])) continue;
                                }
                                partial = false;
                                uint32_t si = sc_index(S[r], N[r], S[r + 1], N[r + 1], S[r + 2], N[r + 2], x);
                                uint32_t e = L.sc[si];
                                uint32_t sg = mq_decode(q, L, CTX_SC + (e & 15)) ^ (e >> 4);
                                S[r + 1] |= bx;
                                if (sg) N[r + 1] |= bx;
                                BT[r] |= bx;
                                PI[r] |= bx;      // newly significant in cleanup: coded this plane
                            }
                        }
                        for (uint32_t r = 0; r < nr; ++r) {
                            L.sig[k + r + 1] = S[r + 1]; L.neg[k + r + 1] = N[r + 1]; L.pi[k + r] = PI[r]; L.bit[k + r] = BT[r];
                        }
                    }
                }
            }
        }
        // broadcast progress
        pt_done = __shfl(pt_done, 0);
        p = __shfl(p, 0);
        LDS_BARRIER();
        int pt_end = first_pt + pt_done;   // passes of this plane processed: [first_pt, pt_end)
        // fold plane bits: samples coded in this plane (newly significant, or refined)
        // pi marks SP-visited; for the fold we need "coded": sig && (bit-touched).  A sample
        // significant before this plane is refined iff the MR pass ran (pt_end >= 2).
        // Newly significant samples (SP or CL) have their bit set in L.bit.
        stale = 0;
#pragma unroll
        for (int y = 0; y < 64; ++y) {
            if (y < (int)h) {
                uint32_t bitv = (uint32_t)((L.bit[y] >> lane) & 1);
                bool was = M[y] != 0;
                bool coded = was ? (pt_end >= 2) : (bitv != 0);
                if (coded) M[y] = (M[y] << 1) | bitv;
                else if (was) stale |= 1ull << y;
            }
        }
        if (pt_end < 3) partial_last = true;
        lastplane = bpno1;
        LDS_BARRIER();
        if (lane == 0) {
            for (uint32_t y = 0; y < h; ++y) {
                L.bit[y] = 0;
                if (pt_end == 3) L.pi[y] = 0;     // cleanup clears visited flags
            }
        }
        LDS_BARRIER();
        if (pt_end == 3) { passtype = 0; --bpno1; } else passtype = pt_end;
        if (partial_last) break;
    }
    // ---- reconstruction and dequantisation
    const bool irrev = B.flags & 1;
    float* fcoef = reinterpret_cast<float*>(coef);
#pragma unroll
    for (int y = 0; y < 64; ++y) {
        if (y < (int)h && lane < (int)w) {
            int32_t v = 0;
            if (M[y]) {
                // Grok's pre-filter value (2M+1) * 2^(lastplane-1), sign applied
                int lp = ((stale >> y) & 1) ? lastplane + 1 : lastplane;
                int32_t mag = (int32_t)((2 * M[y] + 1) << (lp - 1));
                bool ng = (L.neg[y + 1] >> lane) & 1;
                v = ng ? -mag : mag;
            }
            size_t o = B.band_off + (size_t)y * B.stride + lane;
            if (irrev) fcoef[o] = (float)v * B.step;      // ScaleFilter: step = stepsize / 2
            else coef[o] = v / 2;
        }
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

void gk_launch_dc_rct_fwd(hipStream_t st, const int32_t* r, const int32_t* g, const int32_t* b, uint32_t sin,
                          int32_t* y, int32_t* u, int32_t* v, uint32_t sout, uint32_t w, uint32_t h, int32_t shift) {
    dim3 grid((w + 1023) / 1024, h);
    hipLaunchKernelGGL(k_dc_rct_fwd, grid, dim3(256), 0, st, r, g, b, sin, y, u, v, sout, w, h, shift);
}
void gk_launch_dc_fwd(hipStream_t st, const int32_t* in, uint32_t sin, int32_t* out, uint32_t sout, uint32_t w,
                      uint32_t h, int32_t shift) {
    dim3 grid((w + 255) / 256, h);
    hipLaunchKernelGGL(k_dc_fwd, grid, dim3(256), 0, st, in, sin, out, sout, w, h, shift);
}
void gk_launch_rct_inv_dc(hipStream_t st, const int32_t* y, const int32_t* u, const int32_t* v, uint32_t sin,
                          int32_t* r, int32_t* g, int32_t* b, uint32_t sout, uint32_t w, uint32_t h, int32_t shift,
                          int32_t mn, int32_t mx) {
    dim3 grid((w + 1023) / 1024, h);
    hipLaunchKernelGGL(k_rct_inv_dc, grid, dim3(256), 0, st, y, u, v, sin, r, g, b, sout, w, h, shift, mn, mx);
}
void gk_launch_dc_inv(hipStream_t st, const int32_t* in, uint32_t sin, int32_t* out, uint32_t sout, uint32_t w,
                      uint32_t h, int32_t shift, int32_t mn, int32_t mx) {
    dim3 grid((w + 255) / 256, h);
    hipLaunchKernelGGL(k_dc_inv, grid, dim3(256), 0, st, in, sin, out, sout, w, h, shift, mn, mx);
}
void gk_launch_dwt53_fwd(hipStream_t st, const int32_t* src, uint32_t sstride, int32_t* dst, uint32_t dstride,
                         uint32_t w, uint32_t h) {
    dim3 grid((w + DWT_TW - 1) / DWT_TW, (h + DWT_TH - 1) / DWT_TH);
    hipLaunchKernelGGL(k_dwt53_fwd_level, grid, dim3(256), 0, st, src, sstride, dst, dstride, w, h);
}
void gk_launch_dwt53_inv(hipStream_t st, const int32_t* src, uint32_t sstride, int32_t* dst, uint32_t dstride,
                         uint32_t w, uint32_t h) {
    dim3 grid((w + DWT_TW - 1) / DWT_TW, (h + DWT_TH - 1) / DWT_TH);
    hipLaunchKernelGGL(k_dwt53_inv_level, grid, dim3(256), 0, st, src, sstride, dst, dstride, w, h);
}
void gk_launch_t1_encode(hipStream_t st, const int32_t* coef, GkBlock* blocks, uint8_t* bytes, GkPass* passes,
                         uint32_t* info, uint32_t nblocks, int* err) {
    if (!nblocks) return;
    hipLaunchKernelGGL(k_t1_encode, dim3(nblocks), dim3(64), 0, st, coef, blocks, bytes, passes, info, nblocks, err);
}
void gk_launch_t1_decode(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, int32_t* coef,
                         uint32_t nblocks) {
    if (!nblocks) return;
    hipLaunchKernelGGL(k_t1_decode, dim3(nblocks), dim3(64), 0, st, bytes, blocks, coef, nblocks);
}
void gk_launch_gather(hipStream_t st, const uint8_t* src, uint8_t* dst, const uint64_t* seg, uint32_t nseg) {
    if (!nseg) return;
    hipLaunchKernelGGL(k_gather, dim3((nseg + 3) / 4), dim3(256), 0, st, src, dst, seg, nseg);
}
