// gk_t1dec.hip — Part-1 T1 decoder for CDNA4, one lane per code-block.
//
// Decoding is a serial chain per code-block (every MQ decision feeds the next
// context), so the parallelism is the code-blocks themselves: 64 blocks per
// wave, each lane running T1::decompress_cblk (T1.cpp:934-1446) on its own
// block.  Per-stripe state (6 significance rows, 6 sign rows, visited and
// refinement rows) lives in 64-bit registers; the block's persistent row
// bitmaps live in a per-block scratch slab (L2-resident).  Each bit-plane's
// decoded magnitude bits are stored as row bitmaps; k_t1_recon (wave per block,
// lane = column) then rebuilds Grok's pre-filter values (2M+1)<<q and applies
// the ShiftFilter / ScaleFilter dequantisation (filters/PostDecompressFilters.h)
// straight into the band window.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"
#include "gk_t1_common.h"

// scratch layout per block (uint64 words)
#define ST_SIG 0      // 66 rows (row y at index y + 1)
#define ST_NEG 66     // 66 rows
#define ST_MU 132     // 64 rows
#define ST_PI 196     // 64 rows
#define ST_BITS 260   // numbps planes x 64 rows (plane 0 = first decoded plane)

struct MqDec {
    uint32_t a, c, ct;
    uint32_t bp, len;
    const uint8_t* p;       // 16-byte aligned staging of this block's bytes
    uint64_t w0, w1;        // bytes [8*k, 8*k+16) where k = bp >> 3
    uint32_t wk;
};

__device__ __forceinline__ uint32_t dec_byte(const MqDec& q, uint32_t i) {
    if (i >= q.len) return 0xffu;
    uint32_t k = i >> 3;
    uint64_t w = (k == q.wk) ? q.w0 : q.w1;
    return (uint32_t)(w >> (8 * (i & 7))) & 0xffu;
}
__device__ __forceinline__ void dec_advance(MqDec& q) {
    ++q.bp;
    if ((q.bp >> 3) != q.wk) {
        q.wk = q.bp >> 3;
        q.w0 = q.w1;
        q.w1 = *(const uint64_t*)(q.p + 8 * (q.wk + 1));
    }
}
__device__ __forceinline__ void dec_bytein(MqDec& q) {
    uint32_t cur = dec_byte(q, q.bp), nxt = dec_byte(q, q.bp + 1);
    if (cur == 0xff) {
        if (nxt > 0x8f) { q.c += 0xff00; q.ct = 8; }
        else { dec_advance(q); q.c += nxt << 9; q.ct = 7; }
    } else { dec_advance(q); q.c += nxt << 8; q.ct = 8; }
}

struct Ctx5 { uint32_t w[5]; };

__device__ __forceinline__ uint32_t mq_dec(MqDec& q, Ctx5& cw, const uint32_t* tab, uint32_t cx) {
    const uint32_t wi = cx >> 2, shb = (cx & 3) * 8;
    uint32_t word = wi == 0 ? cw.w[0] : wi == 1 ? cw.w[1] : wi == 2 ? cw.w[2] : wi == 3 ? cw.w[3] : cw.w[4];
    const uint32_t st = (word >> shb) & 0xff;
    const uint32_t mps = st >> 6;
    const uint32_t e = tab[st & 63];
    const uint32_t qe = e & 0xffff;
    uint32_t d, nst;
    q.a -= qe;
    if ((q.c >> 16) < qe) {
        if (q.a < qe) { d = mps; nst = ((e >> 16) & 0x3f) | (mps << 6); }
        else { d = mps ^ 1; nst = ((e >> 22) & 0x3f) | ((mps ^ (e >> 28)) << 6); }
        q.a = qe;
    } else {
        q.c -= qe << 16;
        if (q.a & 0x8000) return mps;
        if (q.a < qe) { d = mps ^ 1; nst = ((e >> 22) & 0x3f) | ((mps ^ (e >> 28)) << 6); }
        else { d = mps; nst = ((e >> 16) & 0x3f) | (mps << 6); }
    }
    word = (word & ~(0xffu << shb)) | (nst << shb);
    if (wi == 0) cw.w[0] = word; else if (wi == 1) cw.w[1] = word; else if (wi == 2) cw.w[2] = word;
    else if (wi == 3) cw.w[3] = word; else cw.w[4] = word;
    uint32_t n = __clz(q.a) - 16;
    while (n) {
        if (q.ct == 0) dec_bytein(q);
        uint32_t k = n < q.ct ? n : q.ct;
        q.a <<= k; q.c <<= k; q.ct -= k; n -= k;
    }
    return d;
}

__device__ __forceinline__ uint32_t w3(uint64_t row, uint32_t x) {
    return (uint32_t)((x ? (row >> (x - 1)) : (row << 1)) & 7);
}
__device__ __forceinline__ uint32_t f9(uint64_t up, uint64_t mid, uint64_t dn, uint32_t x) {
    return w3(up, x) | ((w3(mid, x) & 5) << 3) | (w3(dn, x) << 6);
}
__device__ __forceinline__ uint64_t dil(uint64_t u, uint64_t m, uint64_t d) {
    uint64_t t = u | m | d;
    return u | d | (t << 1) | (t >> 1);
}
__device__ __forceinline__ uint32_t scx(uint64_t su, uint64_t nu, uint64_t sm, uint64_t nm, uint64_t sd, uint64_t nd,
                                        uint32_t x) {
    uint32_t wv = x ? (uint32_t)((sm >> (x - 1)) & 1) : 0, wn = x ? (uint32_t)((nm >> (x - 1)) & 1) : 0;
    uint32_t ev = x < 63 ? (uint32_t)((sm >> (x + 1)) & 1) : 0, en = x < 63 ? (uint32_t)((nm >> (x + 1)) & 1) : 0;
    uint32_t nv = (uint32_t)((su >> x) & 1), nn = (uint32_t)((nu >> x) & 1);
    uint32_t sv = (uint32_t)((sd >> x) & 1), sn = (uint32_t)((nd >> x) & 1);
    return (wn & wv) | (wv << 1) | ((en & ev) << 2) | (ev << 3) | ((nn & nv) << 4) | (nv << 5) | ((sn & sv) << 6) |
           (sv << 7);
}

struct DecLds {
    uint32_t tab[47];
    uint8_t zc[4][512];
    uint8_t sc[256];
};

// significance decode of one sample (used by SP and CL)
#define SIG_DECODE(UP, MID, DN, NUP, NMID, NDN, BT)                                             \
    {                                                                                           \
        uint32_t e_ = Ls.sc[scx(UP, NUP, MID, NMID, DN, NDN, x)];                               \
        uint32_t sg_ = mq_dec(q, cw, Ls.tab, CTX_SC + (e_ & 15)) ^ (e_ >> 4);                   \
        MID |= bx;                                                                              \
        if (sg_) NMID |= bx;                                                                    \
        BT |= bx;                                                                               \
    }

__global__ __launch_bounds__(64) void k_t1_dec(const uint8_t* __restrict__ bytes, const GkBlock* __restrict__ blocks,
                                               uint64_t* __restrict__ scratch, const uint64_t* __restrict__ st_off,
                                               uint32_t nblocks) {
    __shared__ DecLds Ls;
    const int lane = threadIdx.x;
    if (lane < 47) Ls.tab[lane] = c_mq[lane];
    for (int i = lane; i < 2048; i += 64) Ls.zc[i >> 9][i & 511] = zc_rule((uint32_t)(i >> 9), (uint32_t)(i & 511));
    for (int i = lane; i < 256; i += 64) Ls.sc[i] = sc_rule((uint32_t)i);
    __syncthreads();
    const uint32_t b = blockIdx.x * 64 + lane;
    if (b >= nblocks) return;
    const GkBlock B = blocks[b];
    const uint32_t numbps = B.numbps, npasses = B.npasses;
    uint64_t* ST = scratch + st_off[b];
    const uint32_t w = B.w, h = B.h;
    for (int i = 0; i < 260; ++i) ST[i] = 0;
    if (!npasses || !numbps) return;
    const uint8_t* zc = Ls.zc[B.orient];
    const uint64_t colmask = w >= 64 ? ~0ull : ((1ull << w) - 1);
    MqDec q;
    q.p = bytes + B.data_off; q.len = B.len; q.bp = 0; q.wk = 0;
    q.w0 = *(const uint64_t*)(q.p);
    q.w1 = *(const uint64_t*)(q.p + 8);
    q.c = (q.len == 0 ? 0xffu : dec_byte(q, 0)) << 16;
    dec_bytein(q);
    q.c <<= 7; q.ct -= 7; q.a = 0x8000;
    Ctx5 cw;
    cw.w[0] = 4u; cw.w[1] = 0; cw.w[2] = 0; cw.w[3] = 0; cw.w[4] = (3u << 8) | (46u << 16);
    const uint32_t nstripes = (h + 3) >> 2;
    uint32_t pass = 0;
    for (int bpno = (int)numbps - 1; bpno >= 0 && pass < npasses; --bpno) {
        uint64_t* BITS = ST + ST_BITS + (size_t)(numbps - 1 - bpno) * 64;
        const bool first = bpno == (int)numbps - 1;
        if (!first) {
            // ---------------- significance propagation (T1.cpp:1182-1245)
            for (uint32_t s = 0; s < nstripes; ++s) {
                const uint32_t y0 = 4 * s, nr = h - y0 < 4 ? h - y0 : 4;
                uint64_t S0 = ST[ST_SIG + y0], S1 = ST[ST_SIG + y0 + 1], S2 = ST[ST_SIG + y0 + 2],
                         S3 = ST[ST_SIG + y0 + 3], S4 = ST[ST_SIG + y0 + 4], S5 = ST[ST_SIG + y0 + 5];
                uint64_t N0 = ST[ST_NEG + y0], N1 = ST[ST_NEG + y0 + 1], N2 = ST[ST_NEG + y0 + 2],
                         N3 = ST[ST_NEG + y0 + 3], N4 = ST[ST_NEG + y0 + 4], N5 = ST[ST_NEG + y0 + 5];
                uint64_t P0 = 0, P1 = nr > 1 ? 0 : ~0ull, P2 = nr > 2 ? 0 : ~0ull, P3 = nr > 3 ? 0 : ~0ull;
                uint64_t B0 = 0, B1 = 0, B2 = 0, B3 = 0;
                uint32_t x = 0;
                while (x < 64) {
                    uint64_t cand = (~S1 & ~P0 & dil(S0, S1, S2)) | (~S2 & ~P1 & dil(S1, S2, S3)) |
                                    (~S3 & ~P2 & dil(S2, S3, S4)) | (~S4 & ~P3 & dil(S3, S4, S5));
                    cand &= colmask & (~0ull << x);
                    if (!cand) break;
                    x = (uint32_t)__ffsll((long long)cand) - 1;
                    const uint64_t bx = 1ull << x;
                    if (!((S1 | P0) & bx)) { uint32_t f = f9(S0, S1, S2, x); if (f) { if (mq_dec(q, cw, Ls.tab, zc[f])) SIG_DECODE(S0, S1, S2, N0, N1, N2, B0); P0 |= bx; } }
                    if (!((S2 | P1) & bx)) { uint32_t f = f9(S1, S2, S3, x); if (f) { if (mq_dec(q, cw, Ls.tab, zc[f])) SIG_DECODE(S1, S2, S3, N1, N2, N3, B1); P1 |= bx; } }
                    if (!((S3 | P2) & bx)) { uint32_t f = f9(S2, S3, S4, x); if (f) { if (mq_dec(q, cw, Ls.tab, zc[f])) SIG_DECODE(S2, S3, S4, N2, N3, N4, B2); P2 |= bx; } }
                    if (!((S4 | P3) & bx)) { uint32_t f = f9(S3, S4, S5, x); if (f) { if (mq_dec(q, cw, Ls.tab, zc[f])) SIG_DECODE(S3, S4, S5, N3, N4, N5, B3); P3 |= bx; } }
                    ++x;
                }
                ST[ST_SIG + y0 + 1] = S1; ST[ST_NEG + y0 + 1] = N1; ST[ST_PI + y0] = P0; BITS[y0] = B0;
                if (nr > 1) { ST[ST_SIG + y0 + 2] = S2; ST[ST_NEG + y0 + 2] = N2; ST[ST_PI + y0 + 1] = P1; BITS[y0 + 1] = B1; }
                if (nr > 2) { ST[ST_SIG + y0 + 3] = S3; ST[ST_NEG + y0 + 3] = N3; ST[ST_PI + y0 + 2] = P2; BITS[y0 + 2] = B2; }
                if (nr > 3) { ST[ST_SIG + y0 + 4] = S4; ST[ST_NEG + y0 + 4] = N4; ST[ST_PI + y0 + 3] = P3; BITS[y0 + 3] = B3; }
            }
            if (++pass >= npasses) break;
            // ---------------- magnitude refinement (T1.cpp:1310-1364)
            for (uint32_t s = 0; s < nstripes; ++s) {
                const uint32_t y0 = 4 * s, nr = h - y0 < 4 ? h - y0 : 4;
                uint64_t S0 = ST[ST_SIG + y0], S1 = ST[ST_SIG + y0 + 1], S2 = ST[ST_SIG + y0 + 2],
                         S3 = ST[ST_SIG + y0 + 3], S4 = ST[ST_SIG + y0 + 4], S5 = ST[ST_SIG + y0 + 5];
                uint64_t M0 = ST[ST_MU + y0], M1 = ST[ST_MU + y0 + 1], M2 = ST[ST_MU + y0 + 2], M3 = ST[ST_MU + y0 + 3];
                uint64_t P0 = ST[ST_PI + y0], P1 = ST[ST_PI + y0 + 1], P2 = ST[ST_PI + y0 + 2], P3 = ST[ST_PI + y0 + 3];
                uint64_t B0 = BITS[y0], B1 = nr > 1 ? BITS[y0 + 1] : 0, B2 = nr > 2 ? BITS[y0 + 2] : 0,
                         B3 = nr > 3 ? BITS[y0 + 3] : 0;
                const uint64_t c0 = S1 & ~P0, c1 = nr > 1 ? S2 & ~P1 : 0, c2 = nr > 2 ? S3 & ~P2 : 0,
                               c3 = nr > 3 ? S4 & ~P3 : 0;
                uint64_t cols = (c0 | c1 | c2 | c3) & colmask;
                while (cols) {
                    const uint32_t x = (uint32_t)__ffsll((long long)cols) - 1;
                    const uint64_t bx = 1ull << x;
                    cols &= cols - 1;
                    if (c0 & bx) { uint32_t cx = (M0 & bx) ? CTX_MAG + 2 : (f9(S0, S1, S2, x) ? CTX_MAG + 1 : CTX_MAG); if (mq_dec(q, cw, Ls.tab, cx)) B0 |= bx; M0 |= bx; }
                    if (c1 & bx) { uint32_t cx = (M1 & bx) ? CTX_MAG + 2 : (f9(S1, S2, S3, x) ? CTX_MAG + 1 : CTX_MAG); if (mq_dec(q, cw, Ls.tab, cx)) B1 |= bx; M1 |= bx; }
                    if (c2 & bx) { uint32_t cx = (M2 & bx) ? CTX_MAG + 2 : (f9(S2, S3, S4, x) ? CTX_MAG + 1 : CTX_MAG); if (mq_dec(q, cw, Ls.tab, cx)) B2 |= bx; M2 |= bx; }
                    if (c3 & bx) { uint32_t cx = (M3 & bx) ? CTX_MAG + 2 : (f9(S3, S4, S5, x) ? CTX_MAG + 1 : CTX_MAG); if (mq_dec(q, cw, Ls.tab, cx)) B3 |= bx; M3 |= bx; }
                }
                ST[ST_MU + y0] = M0; BITS[y0] = B0;
                if (nr > 1) { ST[ST_MU + y0 + 1] = M1; BITS[y0 + 1] = B1; }
                if (nr > 2) { ST[ST_MU + y0 + 2] = M2; BITS[y0 + 2] = B2; }
                if (nr > 3) { ST[ST_MU + y0 + 3] = M3; BITS[y0 + 3] = B3; }
            }
            if (++pass >= npasses) break;
        }
        // ---------------- cleanup (T1.cpp:974-1093)
        for (uint32_t s = 0; s < nstripes; ++s) {
            const uint32_t y0 = 4 * s, nr = h - y0 < 4 ? h - y0 : 4;
            uint64_t S0 = ST[ST_SIG + y0], S1 = ST[ST_SIG + y0 + 1], S2 = ST[ST_SIG + y0 + 2],
                     S3 = ST[ST_SIG + y0 + 3], S4 = ST[ST_SIG + y0 + 4], S5 = ST[ST_SIG + y0 + 5];
            uint64_t N0 = ST[ST_NEG + y0], N1 = ST[ST_NEG + y0 + 1], N2 = ST[ST_NEG + y0 + 2],
                     N3 = ST[ST_NEG + y0 + 3], N4 = ST[ST_NEG + y0 + 4], N5 = ST[ST_NEG + y0 + 5];
            uint64_t P0 = first ? 0 : ST[ST_PI + y0];
            uint64_t P1 = nr > 1 ? (first ? 0 : ST[ST_PI + y0 + 1]) : ~0ull;
            uint64_t P2 = nr > 2 ? (first ? 0 : ST[ST_PI + y0 + 2]) : ~0ull;
            uint64_t P3 = nr > 3 ? (first ? 0 : ST[ST_PI + y0 + 3]) : ~0ull;
            uint64_t B0 = first ? 0 : BITS[y0], B1 = (nr > 1 && !first) ? BITS[y0 + 1] : 0,
                     B2 = (nr > 2 && !first) ? BITS[y0 + 2] : 0, B3 = (nr > 3 && !first) ? BITS[y0 + 3] : 0;
            uint64_t cols = ((~S1 & ~P0) | (~S2 & ~P1) | (~S3 & ~P2) | (~S4 & ~P3)) & colmask;
            while (cols) {
                const uint32_t x = (uint32_t)__ffsll((long long)cols) - 1;
                const uint64_t bx = 1ull << x;
                cols &= cols - 1;
                uint32_t start = 0;
                if (nr == 4 && !((S1 | S2 | S3 | S4 | P0 | P1 | P2 | P3) & bx) && !f9(S0, S1, S2, x) &&
                    !f9(S1, S2, S3, x) && !f9(S2, S3, S4, x) && !f9(S3, S4, S5, x)) {
                    // run-length mode
                    if (!mq_dec(q, cw, Ls.tab, CTX_AGG)) continue;
                    uint32_t rl = mq_dec(q, cw, Ls.tab, CTX_UNI);
                    rl = (rl << 1) | mq_dec(q, cw, Ls.tab, CTX_UNI);
                    if (rl == 0) SIG_DECODE(S0, S1, S2, N0, N1, N2, B0)
                    else if (rl == 1) SIG_DECODE(S1, S2, S3, N1, N2, N3, B1)
                    else if (rl == 2) SIG_DECODE(S2, S3, S4, N2, N3, N4, B2)
                    else SIG_DECODE(S3, S4, S5, N3, N4, N5, B3)
                    start = rl + 1;
                }
                if (start <= 0 && !((S1 | P0) & bx)) { if (mq_dec(q, cw, Ls.tab, zc[f9(S0, S1, S2, x)])) SIG_DECODE(S0, S1, S2, N0, N1, N2, B0); }
                if (start <= 1 && !((S2 | P1) & bx)) { if (mq_dec(q, cw, Ls.tab, zc[f9(S1, S2, S3, x)])) SIG_DECODE(S1, S2, S3, N1, N2, N3, B1); }
                if (start <= 2 && !((S3 | P2) & bx)) { if (mq_dec(q, cw, Ls.tab, zc[f9(S2, S3, S4, x)])) SIG_DECODE(S2, S3, S4, N2, N3, N4, B2); }
                if (start <= 3 && !((S4 | P3) & bx)) { if (mq_dec(q, cw, Ls.tab, zc[f9(S3, S4, S5, x)])) SIG_DECODE(S3, S4, S5, N3, N4, N5, B3); }
            }
            ST[ST_SIG + y0 + 1] = S1; ST[ST_NEG + y0 + 1] = N1; BITS[y0] = B0;
            if (nr > 1) { ST[ST_SIG + y0 + 2] = S2; ST[ST_NEG + y0 + 2] = N2; BITS[y0 + 1] = B1; }
            if (nr > 2) { ST[ST_SIG + y0 + 3] = S3; ST[ST_NEG + y0 + 3] = N3; BITS[y0 + 2] = B2; }
            if (nr > 3) { ST[ST_SIG + y0 + 4] = S4; ST[ST_NEG + y0 + 4] = N4; BITS[y0 + 3] = B3; }
        }
        ++pass;
    }
}

// Reconstruction + dequantisation: wave per block, lane = column.
__global__ __launch_bounds__(64) void k_t1_recon(const GkBlock* __restrict__ blocks,
                                                 const uint64_t* __restrict__ scratch,
                                                 const uint64_t* __restrict__ st_off, int32_t* __restrict__ coef,
                                                 uint32_t nblocks) {
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const int x = threadIdx.x;
    const GkBlock B = blocks[b];
    if (x >= (int)B.w) return;
    const uint64_t* ST = scratch + st_off[b];
    const bool irrev = B.flags & 1;
    float* fcoef = reinterpret_cast<float*>(coef);
    const uint32_t numbps = B.numbps, npasses = B.npasses;
    // last decoded pass: k = npasses-1; pass k>0 belongs to plane P0-(k+2)/3, type (k+2)%3
    int bpl = 0, t = 2;
    if (npasses && numbps) {
        int k = (int)npasses - 1;
        if (k > 3 * (int)numbps - 3) k = 3 * (int)numbps - 3;
        bpl = (int)numbps - 1 - (k + 2) / 3;
        t = (k + 2) % 3;
    }
    for (uint32_t y = 0; y < B.h; ++y) {
        int32_t v = 0;
        if (npasses && numbps) {
            uint32_t M = 0;
            for (int p = (int)numbps - 1; p >= bpl; --p) {
                uint64_t row = ST[ST_BITS + (size_t)(numbps - 1 - p) * 64 + y];
                M |= (uint32_t)((row >> x) & 1) << p;
            }
            if (M) {
                int qq = (t == 0 && (M >> (bpl + 1)) != 0) ? bpl + 1 : bpl;
                int32_t mag = (int32_t)(((M >> qq) << 1 | 1) << qq);
                bool ng = (ST[ST_NEG + y + 1] >> x) & 1;
                v = ng ? -mag : mag;
            }
        }
        size_t o = B.band_off + (size_t)y * B.stride + x;
        if (irrev) fcoef[o] = (float)v * B.step;
        else coef[o] = v / 2;
    }
}

#include "gk_launch.h"
void gk_launch_t1_dec(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, uint64_t* scratch,
                      const uint64_t* st_off, uint32_t nblocks) {
    if (!nblocks) return;
    hipLaunchKernelGGL(k_t1_dec, dim3((nblocks + 63) / 64), dim3(64), 0, st, bytes, blocks, scratch, st_off, nblocks);
}
void gk_launch_t1_recon(hipStream_t st, const GkBlock* blocks, const uint64_t* scratch, const uint64_t* st_off,
                        int32_t* coef, uint32_t nblocks) {
    if (!nblocks) return;
    hipLaunchKernelGGL(k_t1_recon, dim3(nblocks), dim3(64), 0, st, blocks, scratch, st_off, coef, nblocks);
}
