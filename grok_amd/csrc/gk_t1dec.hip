// gk_t1dec.hip — Part-1 T1 decoder for CDNA4: one lane per code-block,
// stripe-synchronous waves.
//
// Decoding is a serial chain per code-block (every MQ decision feeds the next
// context; T1::decompress_cblk, T1.cpp:934-1446), so the parallelism is the
// code-blocks: each lane of a wave decodes its own block.  To keep the 64
// chains of a wave convergent, all lanes walk the same (bit-plane, pass,
// stripe) sequence and, inside a stripe-pass, advance in lock-step *steps*:
// every step each lane locates its next coding position, forms the context and
// decodes exactly one MQ symbol.  Control flow is uniform per step; only data
// differs between lanes.
//
// Per-lane stripe state (significance / sign / visited / refined / plane-bit
// rows as 64-bit column masks) lives in VGPRs while a stripe is processed and
// in a per-wave scratch slab between passes, laid out [row][lane] so every
// stripe load/store is one coalesced 512-byte access.  The compressed bytes
// stream through a 32-byte per-lane register window refilled at uniform step
// intervals with a 16-byte look-ahead load, so no lane waits on memory inside
// a step.  Blocks are assigned to lanes sorted by pass count (host), so the
// lanes of a wave carry similar work.
//
// k_t1_recon (wave per block, lane = column) rebuilds Grok's pre-filter values
// (2M+1)<<q from the decoded bit-planes and applies ShiftFilter / ScaleFilter
// (filters/PostDecompressFilters.h) straight into the band window.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"
#include "gk_t1_common.h"
#include <cstdio>
#include <cstdlib>

// per-wave scratch (uint64 words), row r of field F at (F + r) * 64 + lane
#define WS_SIG 0      // 66 rows (row y at y + 1, guards 0 and 65)
#define WS_NEG 66     // 66 rows
#define WS_MU 132     // 64 rows: refined in an earlier plane
#define WS_PI 196     // 64 rows: visited in the current plane
#define WS_BITS 260   // numbps planes x 64 rows: bit of the plane (plane 0 = most significant)
#define WS_FIXED 260

// ------------------------------------------------------------------ MQ decoder
// Compressed bytes reach the coder through a 128-byte per-lane ring in LDS
// (dword-interleaved [dword][lane], conflict-free).  Refills happen only at
// stripe-pass boundaries (uniform points outside the step loop): the 32 bytes
// staged in VGPRs by the previous boundary are written and the next 32 are
// requested, so no step waits on global memory.  A lane whose ring runs low
// inside a very dense stripe-pass takes a synchronous top-up (rare).  At the
// end of every step each lane reads the 4 bytes at its position (nb4) from the
// ring, so BYTEIN itself never touches memory.
#define RING_DW 32
struct MqDec {
    uint32_t a, c, ct;
    uint32_t bp, len, fill;      // read position, block length, ring fill position (multiple of 16)
    uint32_t nb4;                // bytes [bp, bp + 4)
    uint32_t sbase;              // staged bytes cover [sbase, sbase + 32)
    uint32_t T0, T1, T2, T3, T4, T5, T6, T7;
    const uint8_t* p;            // block bytes (16-byte aligned slot, padded)
};

__device__ __forceinline__ uint32_t vsel(bool c, uint32_t a, uint32_t b) {
    // per-lane select through v_cndmask, as inline asm so the optimiser cannot turn a
    // select tree over struct fields into a dynamically indexed (scratch) access
    uint64_t m = __ballot(c);
    uint32_t r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}

// bytes at or past the block length read as 0xFF (the MQ decoder's end-of-data rule,
// mqc_dec.cpp BYTEIN), so the per-step byte fetch needs no length test
__device__ __forceinline__ uint32_t ff_past(uint32_t v, uint32_t at, uint32_t len) {
    const int k = (int)len - (int)at;
    return k <= 0 ? 0xffffffffu : (k >= 4 ? v : (v | (0xffffffffu << (8 * k))));
}
__device__ __forceinline__ void ring_write16(uint32_t (*ring)[64], int lane, uint32_t pos, uint32_t a, uint32_t b,
                                             uint32_t c, uint32_t d, uint32_t len) {
    a = ff_past(a, pos, len); b = ff_past(b, pos + 4, len); c = ff_past(c, pos + 8, len); d = ff_past(d, pos + 12, len);
    const uint32_t j = (pos >> 2) & (RING_DW - 1);
    ring[j][lane] = a; ring[j + 1][lane] = b; ring[j + 2][lane] = c; ring[j + 3][lane] = d;
    if (j == 0) ring[RING_DW][lane] = a;   // mirror for wrap-around reads
}
__device__ __forceinline__ uint32_t ring_get4(uint32_t (*ring)[64], int lane, uint32_t bp) {
    const uint32_t j = (bp >> 2) & (RING_DW - 1);
    return __builtin_amdgcn_alignbyte(ring[j + 1][lane], ring[j][lane], bp & 3);
}
template <class Q> __device__ __forceinline__ void stage_load(Q& q) {
    uint4 a = *(const uint4*)(q.p + q.sbase), b = *(const uint4*)(q.p + q.sbase + 16);
    q.T0 = a.x; q.T1 = a.y; q.T2 = a.z; q.T3 = a.w; q.T4 = b.x; q.T5 = b.y; q.T6 = b.z; q.T7 = b.w;
}
// stripe-pass boundary: commit the staged 32 bytes when the ring has room, request the next 32
template <class Q> __device__ __forceinline__ void ring_boundary(uint32_t (*ring)[64], int lane, Q& q) {
    if (q.sbase != q.fill) { q.sbase = q.fill; stage_load(q); }   // after a synchronous top-up
    if (q.fill + 32 - q.bp <= 4 * RING_DW) {
        ring_write16(ring, lane, q.fill, q.T0, q.T1, q.T2, q.T3, q.len);
        ring_write16(ring, lane, q.fill + 16, q.T4, q.T5, q.T6, q.T7, q.len);
        q.fill += 32;
        q.sbase = q.fill;
        stage_load(q);
    }
}
// inside a step loop: synchronous top-up for a lane about to run dry
template <class Q> __device__ __forceinline__ void ring_topup(uint32_t (*ring)[64], int lane, Q& q) {
    if (q.fill - q.bp < 8) {
        uint4 a = *(const uint4*)(q.p + q.fill);
        ring_write16(ring, lane, q.fill, a.x, a.y, a.z, a.w, q.len);
        q.fill += 16;
    }
}

// BYTEIN (mqc_dec.cpp, Annex C.3.4), branch-free: bytes past the end read as 0xFF.
__device__ __forceinline__ void mq_bytein(MqDec& q, bool en) {
    const uint32_t cur = q.bp < q.len ? (q.nb4 & 0xff) : 0xffu;
    const uint32_t nxt = q.bp + 1 < q.len ? ((q.nb4 >> 8) & 0xff) : 0xffu;
    const bool ff = cur == 0xff, stuck = ff && nxt > 0x8f;
    const uint32_t add = stuck ? 0xff00u : (nxt << (ff ? 9 : 8));
    const bool adv = en && !stuck;
    q.c += en ? add : 0u;
    q.ct = en ? ((ff && !stuck) ? 7u : 8u) : q.ct;
    q.bp += adv ? 1u : 0u;
    q.nb4 = adv ? (q.nb4 >> 8) : q.nb4;
}

struct Ctx5 { uint32_t w0, w1, w2, w3, w4; };   // one byte per context: state | mps << 6

// DECODE (Annex C.3.2) for context cx; `en` predicates every state change.
__device__ __forceinline__ uint32_t mq_decode(MqDec& q, Ctx5& cw, const uint32_t* tab, uint32_t cx, bool en) {
    const uint32_t wi = cx >> 2, shb = (cx & 3) * 8;
    uint32_t word = vsel(wi == 4, cw.w4, vsel(wi & 2, vsel(wi & 1, cw.w3, cw.w2), vsel(wi & 1, cw.w1, cw.w0)));
    const uint32_t st = (word >> shb) & 0xff;
    const uint32_t mps = st >> 6;
    const uint32_t e = tab[st & 63];
    const uint32_t qe = e & 0xffff;
    const uint32_t a1 = q.a - qe;
    const bool lower = (q.c >> 16) < qe;
    const bool fast = !lower && (a1 & 0x8000);            // MPS, no renormalisation
    const bool mps_path = lower ? (a1 < qe) : (a1 >= qe);  // exchange rule
    const uint32_t d = (fast || mps_path) ? mps : (mps ^ 1);
    const uint32_t nst = mps_path ? (((e >> 16) & 0x3f) | (mps << 6)) : (((e >> 22) & 0x3f) | ((mps ^ (e >> 28)) << 6));
    const bool upd = en && !fast;
    q.a = en ? (lower ? qe : a1) : q.a;
    q.c = (en && !lower) ? q.c - (qe << 16) : q.c;
    word = (word & ~(0xffu << shb)) | (nst << shb);
    cw.w0 = vsel(upd && wi == 0, word, cw.w0); cw.w1 = vsel(upd && wi == 1, word, cw.w1);
    cw.w2 = vsel(upd && wi == 2, word, cw.w2); cw.w3 = vsel(upd && wi == 3, word, cw.w3);
    cw.w4 = vsel(upd && wi == 4, word, cw.w4);
    // RENORMD: shift n bits, BYTEIN whenever ct reaches 0 before a shift
    uint32_t n = upd ? __clz(q.a) - 16 : 0u;
    while (__any(n != 0)) {
        const bool need = n != 0;
        mq_bytein(q, need && q.ct == 0);
        const uint32_t k = n < q.ct ? n : q.ct;
        q.a <<= k; q.c <<= k; q.ct -= k; n -= k;
    }
    return d;
}

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint64_t dil3(uint64_t u, uint64_t m, uint64_t d) {
    uint64_t t = u | m | d;
    return t | (t << 1) | (t >> 1);
}
// 3-bit window (x-1, x, x+1) of a row
__device__ __forceinline__ uint32_t win3(uint64_t row, uint32_t x) {
    return (uint32_t)((x ? (row >> (x - 1)) : (row << 1)) & 7u);
}
// 18-bit window of six rows: row i -> bits [3i, 3i+3)
__device__ __forceinline__ uint32_t win18(uint64_t r0, uint64_t r1, uint64_t r2, uint64_t r3, uint64_t r4, uint64_t r5,
                                          uint32_t x) {
    return win3(r0, x) | (win3(r1, x) << 3) | (win3(r2, x) << 6) | (win3(r3, x) << 9) | (win3(r4, x) << 12) |
           (win3(r5, x) << 15);
}
// bits of the four stripe rows at column x (bit r = row r)
__device__ __forceinline__ uint32_t col4(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint32_t x) {
    return (uint32_t)((a >> x) & 1) | ((uint32_t)((b >> x) & 1) << 1) | ((uint32_t)((c >> x) & 1) << 2) |
           ((uint32_t)((d >> x) & 1) << 3);
}
// next coding position >= (x, r) in stripe scan order (column-major, rows 0..3);
// returns false when the stripe has none.
__device__ __forceinline__ bool next_pos(uint64_t c0, uint64_t c1, uint64_t c2, uint64_t c3, uint32_t& x, uint32_t& r) {
    if (x < 64) {
        uint32_t m = col4(c0, c1, c2, c3, x) & (0xfu << r);
        if (m) { r = __ffs(m) - 1; return true; }
    }
    uint64_t any = c0 | c1 | c2 | c3;
    any = (x >= 63) ? 0ull : (any & (~0ull << (x + 1)));
    if (!any) return false;
    x = (uint32_t)__ffsll((long long)any) - 1;
    r = __ffs(col4(c0, c1, c2, c3, x)) - 1;
    return true;
}
// sign-context index (bit0 W-neg bit1 W-sig bit2 E-neg bit3 E-sig bit4 N-neg bit5 N-sig bit6 S-neg bit7 S-sig)
// from the 9-bit significance / sign neighbourhoods fs / fn of the sample
__device__ __forceinline__ uint32_t sc_from9(uint32_t fs, uint32_t fn) {
    uint32_t wv = (fs >> 3) & 1, ev = (fs >> 5) & 1, nv = (fs >> 1) & 1, sv = (fs >> 7) & 1;
    uint32_t wn = (fn >> 3) & wv, en = (fn >> 5) & ev, nn = (fn >> 1) & nv, sn = (fn >> 7) & sv;
    return wn | (wv << 1) | (en << 2) | (ev << 3) | (nn << 4) | (nv << 5) | (sn << 6) | (sv << 7);
}
__device__ __forceinline__ uint64_t rowsel(uint32_t r, uint32_t i, uint64_t v) { return r == i ? v : 0ull; }

struct DecLds {
    uint32_t tab[47];
    uint8_t zc[4][512];
    uint8_t sc[256];
    uint32_t ring[RING_DW + 1][64];
};

enum { PH_FIND = 0, PH_SIGN = 1, PH_UNI1 = 2, PH_UNI2 = 3 };

// Everything one lane carries across stripe-passes.
struct LaneDec {
    MqDec q;
    Ctx5 cw;
    uint32_t step;
    uint32_t nsym;
};

__device__ __forceinline__ void step_refill(LaneDec& L, uint32_t (*ring)[64], int lane) {
    ++L.step;
    if (__any(L.q.fill - L.q.bp < 8)) ring_topup(ring, lane, L.q);
}
__device__ __forceinline__ void step_prefetch(LaneDec& L, uint32_t (*ring)[64], int lane) {
    L.q.nb4 = ring_get4(ring, lane, L.q.bp);
}

// Branch-free next coding position >= (x, r) (column-major, rows 0..3).  Returns
// false (x, r unchanged) when the stripe has no further position.
__device__ __forceinline__ bool find_next(uint64_t c0, uint64_t c1, uint64_t c2, uint64_t c3, uint32_t& x, uint32_t& r) {
    const uint32_t xc = x & 63;
    const uint32_t m = (x < 64) ? (col4(c0, c1, c2, c3, xc) & (0xfu << r)) : 0u;
    const uint64_t any = (x >= 63) ? 0ull : ((c0 | c1 | c2 | c3) & (~0ull << (x + 1)));
    const uint32_t xn = (uint32_t)__ffsll((long long)any) - 1;
    const uint32_t mn = col4(c0, c1, c2, c3, xn & 63);
    const bool here = m != 0, found = here || any != 0;
    x = here ? x : (found ? xn : x);
    r = here ? (uint32_t)(__ffs(m) - 1) : (found ? (uint32_t)(__ffs(mn) - 1) : r);
    return found;
}
__device__ __forceinline__ uint64_t rsel(uint32_t r, uint32_t i, uint64_t v) { return r == i ? v : 0ull; }

// ---- significance propagation on one stripe (T1.cpp:1182-1245)
__device__ __forceinline__ void pass_sp(LaneDec& L, DecLds& Ls, const uint8_t* zc, int lane, bool on,
                                        uint64_t S0, uint64_t& S1, uint64_t& S2, uint64_t& S3, uint64_t& S4, uint64_t S5,
                                        uint64_t N0, uint64_t& N1, uint64_t& N2, uint64_t& N3, uint64_t& N4, uint64_t N5,
                                        uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3, uint64_t& P0, uint64_t& P1,
                                        uint64_t& P2, uint64_t& P3) {
    uint64_t C0 = ~S1 & dil3(S0, S1, S2) & v0, C1 = ~S2 & dil3(S1, S2, S3) & v1;
    uint64_t C2 = ~S3 & dil3(S2, S3, S4) & v2, C3 = ~S4 & dil3(S3, S4, S5) & v3;
    uint32_t x = 0, r = 0;
    bool sign = false, pend = on;
    while (__any(pend)) {
        step_refill(L, Ls.ring, lane);
        if (!sign) pend = pend && find_next(C0, C1, C2, C3, x, r);
        const uint32_t sh = 3 * r;
        const uint32_t fs = (win18(S0, S1, S2, S3, S4, S5, x & 63) >> sh) & 0x1ff;
        const uint32_t fn = (win18(N0, N1, N2, N3, N4, N5, x & 63) >> sh) & 0x1ff;
        const uint32_t sce = Ls.sc[sc_from9(fs, fn)];
        const uint32_t cx = sign ? CTX_SC + (sce & 15) : CTX_ZC + zc[fs];
        const uint32_t d = mq_decode(L.q, L.cw, Ls.tab, cx, pend);
        L.nsym += pend ? 1 : 0;
        // sign decoded: the sample becomes significant
        const bool sig = pend && sign;
        const uint64_t bx = sig ? (1ull << (x & 63)) : 0ull, bn = bx << 1;
        const uint64_t m0 = rsel(r, 0, bx), m1 = rsel(r, 1, bx), m2 = rsel(r, 2, bx), m3 = rsel(r, 3, bx);
        S1 |= m0; S2 |= m1; S3 |= m2; S4 |= m3;
        const uint64_t ng = (d ^ (sce >> 4)) ? ~0ull : 0ull;
        N1 |= m0 & ng; N2 |= m1 & ng; N3 |= m2 & ng; N4 |= m3 & ng;
        // later positions that gain a significant neighbour: (x, r+1) and column x+1 rows r-1..r+1
        const uint64_t b0 = rsel(r, 0, bn), b1 = rsel(r, 1, bn), b2 = rsel(r, 2, bn), b3 = rsel(r, 3, bn);
        C0 |= (b0 | b1) & ~S1 & v0;
        C1 |= (m0 | b0 | b1 | b2) & ~S2 & v1;
        C2 |= (m1 | b1 | b2 | b3) & ~S3 & v2;
        C3 |= (m2 | b2 | b3) & ~S4 & v3;
        // advance: after a zero ZC decision or a sign, move to the next row
        const bool adv = pend && (sign || !d);
        sign = pend && !sign && d;
        r += adv ? 1 : 0;
        x += (r == 4) ? 1 : 0;
        r &= 3;
        step_prefetch(L, Ls.ring, lane);
    }
    // every candidate was visited and no visited position was added afterwards: visited = candidates
    P0 = C0; P1 = C1; P2 = C2; P3 = C3;
}

// ---- magnitude refinement on one stripe (T1.cpp:1310-1364)
__device__ __forceinline__ void pass_mr(LaneDec& L, DecLds& Ls, int lane, bool on, uint64_t S0, uint64_t S1, uint64_t S2,
                                        uint64_t S3, uint64_t S4, uint64_t S5, uint64_t v0, uint64_t v1, uint64_t v2,
                                        uint64_t v3, uint64_t P0, uint64_t P1, uint64_t P2, uint64_t P3, uint64_t& M0,
                                        uint64_t& M1, uint64_t& M2, uint64_t& M3, uint64_t& B0, uint64_t& B1,
                                        uint64_t& B2, uint64_t& B3) {
    const uint64_t C0 = S1 & ~P0 & v0, C1 = S2 & ~P1 & v1, C2 = S3 & ~P2 & v2, C3 = S4 & ~P3 & v3;
    uint32_t x = 0, r = 0;
    bool pend = on;
    while (__any(pend)) {
        step_refill(L, Ls.ring, lane);
        pend = pend && find_next(C0, C1, C2, C3, x, r);
        const uint32_t xc = x & 63;
        const uint32_t fs = (win18(S0, S1, S2, S3, S4, S5, xc) >> (3 * r)) & 0x1ef;
        const uint64_t mu = rsel(r, 0, M0) | rsel(r, 1, M1) | rsel(r, 2, M2) | rsel(r, 3, M3);
        const uint32_t cx = ((mu >> xc) & 1) ? CTX_MAG + 2 : (fs ? CTX_MAG + 1 : CTX_MAG);
        const uint32_t d = mq_decode(L.q, L.cw, Ls.tab, cx, pend);
        L.nsym += pend ? 1 : 0;
        const uint64_t bx = (pend && d) ? (1ull << xc) : 0ull;
        B0 |= rsel(r, 0, bx); B1 |= rsel(r, 1, bx); B2 |= rsel(r, 2, bx); B3 |= rsel(r, 3, bx);
        r += pend ? 1 : 0;
        x += (r == 4) ? 1 : 0;
        r &= 3;
        step_prefetch(L, Ls.ring, lane);
    }
    M0 |= C0; M1 |= C1; M2 |= C2; M3 |= C3;   // everything coded here is now refined
}

// ---- cleanup on one stripe (T1.cpp:974-1093)
__device__ __forceinline__ void pass_cl(LaneDec& L, DecLds& Ls, const uint8_t* zc, int lane, bool on, uint32_t nr,
                                        uint64_t S0, uint64_t& S1, uint64_t& S2, uint64_t& S3, uint64_t& S4, uint64_t S5,
                                        uint64_t N0, uint64_t& N1, uint64_t& N2, uint64_t& N3, uint64_t& N4, uint64_t N5,
                                        uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3, uint64_t P0, uint64_t P1,
                                        uint64_t P2, uint64_t P3) {
    const uint64_t C0 = ~S1 & ~P0 & v0, C1 = ~S2 & ~P1 & v1, C2 = ~S3 & ~P2 & v2, C3 = ~S4 & ~P3 & v3;
    // run-length candidates: four coding positions, no significant neighbour at pass start
    const uint64_t E = (nr == 4) ? (C0 & C1 & C2 & C3 & ~dil3(S0 | S1, S2 | S3, S4 | S5)) : 0ull;
    uint64_t fresh = 0;   // samples that became significant during this pass
    uint32_t x = 0, r = 0, ph = PH_FIND, colx = 0xffffffffu, rlhi = 0;
    bool pend = on;
    while (__any(pend)) {
        step_refill(L, Ls.ring, lane);
        const bool finding = ph == PH_FIND;
        if (finding) pend = pend && find_next(C0, C1, C2, C3, x, r);
        const uint32_t xc = x & 63;
        // a new column starts in run-length mode when it was eligible at pass start and its
        // left neighbour column gained no significance in this pass
        const bool agg = finding && x != colx && ((E >> xc) & 1) && !(xc && ((fresh >> (xc - 1)) & 1));
        colx = finding ? x : colx;
        const uint32_t sh = 3 * r;
        const uint32_t fs = (win18(S0, S1, S2, S3, S4, S5, xc) >> sh) & 0x1ff;
        const uint32_t fn = (win18(N0, N1, N2, N3, N4, N5, xc) >> sh) & 0x1ff;
        const uint32_t sce = Ls.sc[sc_from9(fs, fn)];
        const uint32_t cx = agg ? CTX_AGG : (ph == PH_SIGN ? CTX_SC + (sce & 15) : (finding ? CTX_ZC + zc[fs] : CTX_UNI));
        const uint32_t d = mq_decode(L.q, L.cw, Ls.tab, cx, pend);
        L.nsym += pend ? 1 : 0;
        const bool sig = pend && ph == PH_SIGN;
        const uint64_t bx = sig ? (1ull << xc) : 0ull;
        const uint64_t m0 = rsel(r, 0, bx), m1 = rsel(r, 1, bx), m2 = rsel(r, 2, bx), m3 = rsel(r, 3, bx);
        S1 |= m0; S2 |= m1; S3 |= m2; S4 |= m3;
        const uint64_t ng = (d ^ (sce >> 4)) ? ~0ull : 0ull;
        N1 |= m0 & ng; N2 |= m1 & ng; N3 |= m2 & ng; N4 |= m3 & ng;
        fresh |= bx;
        // phase transitions
        uint32_t nph = ph, nr2 = r;
        bool col_done = false;
        if (agg) { nph = d ? PH_UNI1 : PH_FIND; col_done = !d; }
        else if (finding) { nph = d ? PH_SIGN : PH_FIND; nr2 = d ? r : r + 1; }
        else if (ph == PH_UNI1) { rlhi = d; nph = PH_UNI2; }
        else if (ph == PH_UNI2) { nr2 = (rlhi << 1) | d; nph = PH_SIGN; }
        else { nph = PH_FIND; nr2 = r + 1; }
        if (pend) {
            ph = nph;
            r = col_done ? 0 : nr2;
            x += (col_done || r == 4) ? 1 : 0;
            r &= 3;
        }
        step_prefetch(L, Ls.ring, lane);
    }
}

__global__ __launch_bounds__(64) void k_t1_dec(const uint8_t* __restrict__ bytes, const GkBlock* __restrict__ blocks,
                                               const uint32_t* __restrict__ order, uint64_t* __restrict__ scratch,
                                               const uint64_t* __restrict__ wave_off, uint32_t nblocks,
                                               unsigned long long* __restrict__ stats) {
    __shared__ DecLds Ls;
    const int lane = threadIdx.x;
    if (lane < 47) Ls.tab[lane] = c_mq[lane];
    for (int i = lane; i < 2048; i += 64) Ls.zc[i >> 9][i & 511] = zc_rule((uint32_t)(i >> 9), (uint32_t)(i & 511));
    for (int i = lane; i < 256; i += 64) Ls.sc[i] = sc_rule((uint32_t)i);
    const uint32_t slot = blockIdx.x * 64 + lane;
    const uint32_t bid = slot < nblocks ? order[slot] : 0xffffffffu;   // empty slots: 0xffffffff
    const bool has = bid != 0xffffffffu;
    GkBlock B = {};
    if (has) B = blocks[bid];
    uint64_t* WS = scratch + wave_off[blockIdx.x];
    const uint32_t numbps = has ? B.numbps : 0, npasses = (has && B.numbps) ? B.npasses : 0;
    const uint32_t w = B.w, h = B.h;
    const uint64_t colmask = w >= 64 ? ~0ull : ((1ull << w) - 1);
    const uint32_t nstripes = (h + 3) >> 2;
    const uint8_t* zc = Ls.zc[B.orient & 3];
    for (int r = 0; r < WS_FIXED; ++r) WS[r * 64 + lane] = 0;   // clear the state rows (coalesced)
    LaneDec L;
    L.cw = {4u, 0u, 0u, 0u, (3u << 8) | (46u << 16)};   // mqc_resetstates: ZC0=4, AGG=3, UNI=46
    L.step = 0; L.nsym = 0;
    MqDec& q = L.q;
    q.p = npasses ? bytes + B.data_off : bytes;
    q.len = npasses ? B.len : 0;
    q.bp = 0; q.fill = 0; q.sbase = 0;
    stage_load(q);
    __syncthreads();
    ring_boundary(Ls.ring, lane, q);
    q.sbase = q.fill; stage_load(q);
    ring_boundary(Ls.ring, lane, q);
    ring_boundary(Ls.ring, lane, q);
    q.nb4 = ring_get4(Ls.ring, lane, 0);
    // INITDEC (mqc_dec.cpp:98-112)
    q.c = (q.len ? (q.nb4 & 0xff) : 0xffu) << 16;
    mq_bytein(q, true);
    q.c <<= 7; q.ct -= 7; q.a = 0x8000;
    // wave-uniform loop bounds
    uint32_t maxplanes = numbps, maxst = nstripes;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        maxplanes = max(maxplanes, (uint32_t)__shfl_xor((int)maxplanes, o));
        maxst = max(maxst, (uint32_t)__shfl_xor((int)maxst, o));
    }
    for (uint32_t k = 0; k < maxplanes; ++k) {
        uint64_t* BITS = WS + (WS_BITS + (size_t)k * 64) * 64;
        for (uint32_t t = (k == 0 ? 2u : 0u); t < 3; ++t) {
            const uint32_t pidx = k == 0 ? 0 : 1 + 3 * (k - 1) + t;   // pass index within the block
            const bool pass_on = k < numbps && pidx < npasses;
            if (!__any(pass_on)) continue;
            for (uint32_t s = 0; s < maxst; ++s) {
                const bool on = pass_on && s < nstripes;
                ring_boundary(Ls.ring, lane, L.q);
                L.q.nb4 = ring_get4(Ls.ring, lane, L.q.bp);
                const uint32_t y0 = 4 * s;
                const uint32_t nr = on ? min(4u, h - y0) : 0;
                const uint64_t v0 = nr > 0 ? colmask : 0, v1 = nr > 1 ? colmask : 0, v2 = nr > 2 ? colmask : 0,
                               v3 = nr > 3 ? colmask : 0;
                uint64_t S0 = WS[(WS_SIG + y0) * 64 + lane], S1 = WS[(WS_SIG + y0 + 1) * 64 + lane],
                         S2 = WS[(WS_SIG + y0 + 2) * 64 + lane], S3 = WS[(WS_SIG + y0 + 3) * 64 + lane],
                         S4 = WS[(WS_SIG + y0 + 4) * 64 + lane], S5 = WS[(WS_SIG + y0 + 5) * 64 + lane];
                if (t == 0) {
                    uint64_t N0 = WS[(WS_NEG + y0) * 64 + lane], N1 = WS[(WS_NEG + y0 + 1) * 64 + lane],
                             N2 = WS[(WS_NEG + y0 + 2) * 64 + lane], N3 = WS[(WS_NEG + y0 + 3) * 64 + lane],
                             N4 = WS[(WS_NEG + y0 + 4) * 64 + lane], N5 = WS[(WS_NEG + y0 + 5) * 64 + lane];
                    const uint64_t T1s = S1, T2s = S2, T3s = S3, T4s = S4;
                    uint64_t P0, P1, P2, P3;
                    pass_sp(L, Ls, zc, lane, on, S0, S1, S2, S3, S4, S5, N0, N1, N2, N3, N4, N5, v0, v1, v2, v3,
                            P0, P1, P2, P3);
                    if (on) {
                        WS[(WS_SIG + y0 + 1) * 64 + lane] = S1; WS[(WS_SIG + y0 + 2) * 64 + lane] = S2;
                        WS[(WS_SIG + y0 + 3) * 64 + lane] = S3; WS[(WS_SIG + y0 + 4) * 64 + lane] = S4;
                        WS[(WS_NEG + y0 + 1) * 64 + lane] = N1; WS[(WS_NEG + y0 + 2) * 64 + lane] = N2;
                        WS[(WS_NEG + y0 + 3) * 64 + lane] = N3; WS[(WS_NEG + y0 + 4) * 64 + lane] = N4;
                        WS[(WS_PI + y0) * 64 + lane] = P0; WS[(WS_PI + y0 + 1) * 64 + lane] = P1;
                        WS[(WS_PI + y0 + 2) * 64 + lane] = P2; WS[(WS_PI + y0 + 3) * 64 + lane] = P3;
                        // plane bits: the newly significant samples
                        BITS[(y0) * 64 + lane] = S1 & ~T1s; BITS[(y0 + 1) * 64 + lane] = S2 & ~T2s;
                        BITS[(y0 + 2) * 64 + lane] = S3 & ~T3s; BITS[(y0 + 3) * 64 + lane] = S4 & ~T4s;
                    }
                } else if (t == 1) {
                    const uint64_t P0 = WS[(WS_PI + y0) * 64 + lane], P1 = WS[(WS_PI + y0 + 1) * 64 + lane],
                                   P2 = WS[(WS_PI + y0 + 2) * 64 + lane], P3 = WS[(WS_PI + y0 + 3) * 64 + lane];
                    uint64_t M0 = WS[(WS_MU + y0) * 64 + lane], M1 = WS[(WS_MU + y0 + 1) * 64 + lane],
                             M2 = WS[(WS_MU + y0 + 2) * 64 + lane], M3 = WS[(WS_MU + y0 + 3) * 64 + lane];
                    uint64_t B0 = BITS[(y0) * 64 + lane], B1 = BITS[(y0 + 1) * 64 + lane],
                             B2 = BITS[(y0 + 2) * 64 + lane], B3 = BITS[(y0 + 3) * 64 + lane];
                    pass_mr(L, Ls, lane, on, S0, S1, S2, S3, S4, S5, v0, v1, v2, v3, P0, P1, P2, P3, M0, M1, M2, M3,
                            B0, B1, B2, B3);
                    if (on) {
                        WS[(WS_MU + y0) * 64 + lane] = M0; WS[(WS_MU + y0 + 1) * 64 + lane] = M1;
                        WS[(WS_MU + y0 + 2) * 64 + lane] = M2; WS[(WS_MU + y0 + 3) * 64 + lane] = M3;
                        BITS[(y0) * 64 + lane] = B0; BITS[(y0 + 1) * 64 + lane] = B1;
                        BITS[(y0 + 2) * 64 + lane] = B2; BITS[(y0 + 3) * 64 + lane] = B3;
                    }
                } else {
                    uint64_t N0 = WS[(WS_NEG + y0) * 64 + lane], N1 = WS[(WS_NEG + y0 + 1) * 64 + lane],
                             N2 = WS[(WS_NEG + y0 + 2) * 64 + lane], N3 = WS[(WS_NEG + y0 + 3) * 64 + lane],
                             N4 = WS[(WS_NEG + y0 + 4) * 64 + lane], N5 = WS[(WS_NEG + y0 + 5) * 64 + lane];
                    uint64_t P0 = 0, P1 = 0, P2 = 0, P3 = 0, B0 = 0, B1 = 0, B2 = 0, B3 = 0;
                    if (k) {
                        P0 = WS[(WS_PI + y0) * 64 + lane]; P1 = WS[(WS_PI + y0 + 1) * 64 + lane];
                        P2 = WS[(WS_PI + y0 + 2) * 64 + lane]; P3 = WS[(WS_PI + y0 + 3) * 64 + lane];
                        B0 = BITS[(y0) * 64 + lane]; B1 = BITS[(y0 + 1) * 64 + lane];
                        B2 = BITS[(y0 + 2) * 64 + lane]; B3 = BITS[(y0 + 3) * 64 + lane];
                    }
                    const uint64_t T1s = S1, T2s = S2, T3s = S3, T4s = S4;
                    pass_cl(L, Ls, zc, lane, on, nr, S0, S1, S2, S3, S4, S5, N0, N1, N2, N3, N4, N5, v0, v1, v2, v3,
                            P0, P1, P2, P3);
                    if (on) {
                        WS[(WS_SIG + y0 + 1) * 64 + lane] = S1; WS[(WS_SIG + y0 + 2) * 64 + lane] = S2;
                        WS[(WS_SIG + y0 + 3) * 64 + lane] = S3; WS[(WS_SIG + y0 + 4) * 64 + lane] = S4;
                        WS[(WS_NEG + y0 + 1) * 64 + lane] = N1; WS[(WS_NEG + y0 + 2) * 64 + lane] = N2;
                        WS[(WS_NEG + y0 + 3) * 64 + lane] = N3; WS[(WS_NEG + y0 + 4) * 64 + lane] = N4;
                        BITS[(y0) * 64 + lane] = B0 | (S1 & ~T1s); BITS[(y0 + 1) * 64 + lane] = B1 | (S2 & ~T2s);
                        BITS[(y0 + 2) * 64 + lane] = B2 | (S3 & ~T3s); BITS[(y0 + 3) * 64 + lane] = B3 | (S4 & ~T4s);
                    }
                }
            }
        }
    }
    if (stats) {
        unsigned long long tot = L.nsym;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        if (lane == 0) { atomicAdd(&stats[0], (unsigned long long)L.step); atomicAdd(&stats[1], tot);
                         atomicMax(&stats[2], (unsigned long long)L.step); }
    }
}

// =============================================================================
// Lane-independent variant: every lane walks its own (plane, pass, stripe)
// sequence.  A step decodes one MQ decision per active lane, whatever pass type
// the lane is in (SP / MR / CL share the position search, the context
// formation and the CL phase machine).  A lane whose stripe-pass has no further
// coding position parks; parked lanes cross their stripe boundary together once
// `kpark` of them wait (or nothing else is active), which amortises the
// divergent boundary code.  The next stripe's rows are prefetched into VGPRs
// when a stripe starts, so a boundary never waits on memory (blocks of fewer
// than three stripes reload synchronously at pass boundaries — their next
// pass starts with rows still being stored).  Measured by
// tools/t1_simt_stats.py: the critical path drops from the sum over stripes of
// the per-stripe maximum over lanes to roughly the heaviest block.
// =============================================================================
struct Rows22 {   // one stripe's rows: S1..S5 / N1..N5 (rows y0..y0+4), P/M/B (rows y0..y0+3)
    uint64_t s1, s2, s3, s4, s5, n1, n2, n3, n4, n5, p0, p1, p2, p3, m0, m1, m2, m3, b0, b1, b2, b3;
};
__device__ __forceinline__ void load_rows(Rows22& R, const uint64_t* WS, const uint64_t* BITS, int lane, uint32_t y0) {
    const uint64_t* sg = WS + (size_t)(WS_SIG + y0 + 1) * 64 + lane;
    const uint64_t* ng = WS + (size_t)(WS_NEG + y0 + 1) * 64 + lane;
    const uint64_t* pi = WS + (size_t)(WS_PI + y0) * 64 + lane;
    const uint64_t* mu = WS + (size_t)(WS_MU + y0) * 64 + lane;
    const uint64_t* bt = BITS + (size_t)y0 * 64 + lane;
    R.s1 = sg[0]; R.s2 = sg[64]; R.s3 = sg[128]; R.s4 = sg[192]; R.s5 = sg[256];
    R.n1 = ng[0]; R.n2 = ng[64]; R.n3 = ng[128]; R.n4 = ng[192]; R.n5 = ng[256];
    R.p0 = pi[0]; R.p1 = pi[64]; R.p2 = pi[128]; R.p3 = pi[192];
    R.m0 = mu[0]; R.m1 = mu[64]; R.m2 = mu[128]; R.m3 = mu[192];
    R.b0 = bt[0]; R.b1 = bt[64]; R.b2 = bt[128]; R.b3 = bt[192];
}

// next (plane, pass type, stripe) after (k, t, s); pass types 0 SP, 1 MR, 2 CL
__device__ __forceinline__ void next_pos3(uint32_t& k, uint32_t& t, uint32_t& s, uint32_t& pidx, uint32_t ns) {
    if (++s == ns) {
        s = 0; ++pidx;
        if (t == 2) { ++k; t = 0; } else ++t;
    }
}

__global__ __launch_bounds__(64) void k_t1_dec_ind(const uint8_t* __restrict__ bytes, const GkBlock* __restrict__ blocks,
                                                   const uint32_t* __restrict__ order, uint64_t* __restrict__ scratch,
                                                   const uint64_t* __restrict__ wave_off, uint32_t nblocks,
                                                   unsigned long long* __restrict__ stats, uint32_t kpark) {
    __shared__ DecLds Ls;
    const int lane = threadIdx.x;
    if (lane < 47) Ls.tab[lane] = c_mq[lane];
    for (int i = lane; i < 2048; i += 64) Ls.zc[i >> 9][i & 511] = zc_rule((uint32_t)(i >> 9), (uint32_t)(i & 511));
    for (int i = lane; i < 256; i += 64) Ls.sc[i] = sc_rule((uint32_t)i);
    const uint32_t slot = blockIdx.x * 64 + lane;
    const uint32_t bid = slot < nblocks ? order[slot] : 0xffffffffu;   // empty slots: 0xffffffff
    const bool has = bid != 0xffffffffu;
    GkBlock B = {};
    if (has) B = blocks[bid];
    uint64_t* WS = scratch + wave_off[blockIdx.x];
    const uint32_t numbps = has ? B.numbps : 0, npasses = (has && B.numbps) ? B.npasses : 0;
    const uint32_t h = B.h;
    const uint64_t colmask = B.w >= 64 ? ~0ull : ((1ull << B.w) - 1);
    const uint32_t ns = (h + 3) >> 2;
    const uint8_t* zc = Ls.zc[B.orient & 3];
    for (int r = 0; r < WS_FIXED; ++r) WS[r * 64 + lane] = 0;   // clear the state rows (coalesced)
    LaneDec L;
    L.cw = {4u, 0u, 0u, 0u, (3u << 8) | (46u << 16)};   // mqc_resetstates: ZC0=4, AGG=3, UNI=46
    L.step = 0; L.nsym = 0;
    MqDec& q = L.q;
    q.p = npasses ? bytes + B.data_off : bytes;
    q.len = npasses ? B.len : 0;
    q.bp = 0; q.fill = 0; q.sbase = 0;
    stage_load(q);
    __syncthreads();
    ring_boundary(Ls.ring, lane, q);
    q.sbase = q.fill; stage_load(q);
    ring_boundary(Ls.ring, lane, q);
    ring_boundary(Ls.ring, lane, q);
    q.nb4 = ring_get4(Ls.ring, lane, 0);
    q.c = (q.len ? (q.nb4 & 0xff) : 0xffu) << 16;   // INITDEC (mqc_dec.cpp:98-112)
    mq_bytein(q, true);
    q.c <<= 7; q.ct -= 7; q.a = 0x8000;

    // position: plane k (0 = top), pass type t, stripe s, pass index pidx; k = 0 has only CL
    uint32_t k = 0, t = 2, s = 0, pidx = 0;
    bool done = npasses == 0, parked = false;
    // stripe state
    uint64_t S0 = 0, S1 = 0, S2 = 0, S3 = 0, S4 = 0, S5 = 0, N0 = 0, N1 = 0, N2 = 0, N3 = 0, N4 = 0, N5 = 0;
    uint64_t P0 = 0, P1 = 0, P2 = 0, P3 = 0, M0 = 0, M1 = 0, M2 = 0, M3 = 0, B0 = 0, B1 = 0, B2 = 0, B3 = 0;
    uint64_t C0, C1, C2, C3, E, fresh = 0;
    uint32_t nr = min(4u, h), x = 0, r = 0, ph = PH_FIND, colx = 0xffffffffu, rlhi = 0;
    {
        const uint64_t v0 = nr > 0 ? colmask : 0, v1 = nr > 1 ? colmask : 0, v2 = nr > 2 ? colmask : 0,
                       v3 = nr > 3 ? colmask : 0;
        C0 = v0; C1 = v1; C2 = v2; C3 = v3;   // first CL: nothing significant yet
        E = (nr == 4) ? colmask : 0ull;
    }
    // prefetch of the next stripe (always valid: rows a later stripe of the same pass reads are not
    // touched by the current stripe; at a pass change small blocks patch rows from registers)
    Rows22 X = {};
    uint32_t nevents = 0;
    {
        uint32_t k2 = k, t2 = t, s2 = s, p2 = pidx;
        next_pos3(k2, t2, s2, p2, ns);
        if (!done && p2 < npasses && k2 < numbps) load_rows(X, WS, WS + (WS_BITS + (size_t)k2 * 64) * 64, lane, 4 * s2);
    }

    while (__any(!done)) {
        // ---------------- stripe boundary for parked lanes (batched)
        const uint32_t nparked = __popcll(__ballot(parked));
        const uint32_t nactive = __popcll(__ballot(!done && !parked));
        if (nparked && (nparked >= kpark || nactive == 0)) {
            ++nevents;
            // commit the bytes staged at the previous boundary first: they are older than this
            // boundary's stores, so waiting for them does not wait for the stores
            // (only when no synchronous top-up moved the fill point since the bytes were staged)
            if (!done && q.sbase == q.fill && q.fill + 32 - q.bp <= 4 * RING_DW) {
                ring_write16(Ls.ring, lane, q.fill, q.T0, q.T1, q.T2, q.T3, q.len);
                ring_write16(Ls.ring, lane, q.fill + 16, q.T4, q.T5, q.T6, q.T7, q.len);
                q.fill += 32;
            }
            if (parked) {
                parked = false;
                if (t == 0) { P0 = C0; P1 = C1; P2 = C2; P3 = C3; }            // visited = candidates
                else if (t == 1) { M0 |= C0; M1 |= C1; M2 |= C2; M3 |= C3; }    // now refined
                const uint32_t y0 = 4 * s;
                uint64_t* sg = WS + (size_t)(WS_SIG + y0 + 1) * 64 + lane;
                uint64_t* ng = WS + (size_t)(WS_NEG + y0 + 1) * 64 + lane;
                uint64_t* pi = WS + (size_t)(WS_PI + y0) * 64 + lane;
                uint64_t* mu = WS + (size_t)(WS_MU + y0) * 64 + lane;
                uint64_t* bt = WS + (WS_BITS + (size_t)k * 64 + y0) * 64 + lane;
                sg[0] = S1; sg[64] = S2; sg[128] = S3; sg[192] = S4;
                ng[0] = N1; ng[64] = N2; ng[128] = N3; ng[192] = N4;
                pi[0] = P0; pi[64] = P1; pi[128] = P2; pi[192] = P3;
                mu[0] = M0; mu[64] = M1; mu[128] = M2; mu[192] = M3;
                bt[0] = B0; bt[64] = B1; bt[128] = B2; bt[192] = B3;
                const uint32_t ok = k;
                next_pos3(k, t, s, pidx, ns);
                done = pidx >= npasses || k >= numbps;
                // new stripe rows: prefetched, except rows the finished stripe still held in
                // registers when the prefetch was issued (1-stripe blocks: all; 2-stripe blocks at
                // a pass change: row 4 = the finished stripe's first row)
                const bool one = ns == 1, two = ns == 2 && s == 0;
                const uint64_t nS0 = s ? S4 : 0ull, nN0 = s ? N4 : 0ull;
                const uint64_t nS1 = one ? S1 : X.s1, nS2 = one ? S2 : X.s2, nS3 = one ? S3 : X.s3, nS4 = one ? S4 : X.s4;
                const uint64_t nS5 = two ? S1 : X.s5;
                const uint64_t nN1 = one ? N1 : X.n1, nN2 = one ? N2 : X.n2, nN3 = one ? N3 : X.n3, nN4 = one ? N4 : X.n4;
                const uint64_t nN5 = two ? N1 : X.n5;
                const uint64_t nP0 = one ? P0 : X.p0, nP1 = one ? P1 : X.p1, nP2 = one ? P2 : X.p2, nP3 = one ? P3 : X.p3;
                const uint64_t nM0 = one ? M0 : X.m0, nM1 = one ? M1 : X.m1, nM2 = one ? M2 : X.m2, nM3 = one ? M3 : X.m3;
                const bool same_plane = one && ok == k;
                const uint64_t nB0 = same_plane ? B0 : X.b0, nB1 = same_plane ? B1 : X.b1, nB2 = same_plane ? B2 : X.b2,
                               nB3 = same_plane ? B3 : X.b3;
                S0 = nS0; S1 = nS1; S2 = nS2; S3 = nS3; S4 = nS4; S5 = nS5;
                N0 = nN0; N1 = nN1; N2 = nN2; N3 = nN3; N4 = nN4; N5 = nN5;
                const bool newplane = t == 0 || k == 0;
                P0 = t == 0 ? 0ull : nP0; P1 = t == 0 ? 0ull : nP1; P2 = t == 0 ? 0ull : nP2; P3 = t == 0 ? 0ull : nP3;
                M0 = nM0; M1 = nM1; M2 = nM2; M3 = nM3;
                B0 = newplane ? 0ull : nB0; B1 = newplane ? 0ull : nB1; B2 = newplane ? 0ull : nB2;
                B3 = newplane ? 0ull : nB3;
                const uint32_t ny0 = 4 * s;
                nr = done ? 0u : min(4u, h - ny0);
                const uint64_t v0 = nr > 0 ? colmask : 0, v1 = nr > 1 ? colmask : 0, v2 = nr > 2 ? colmask : 0,
                               v3 = nr > 3 ? colmask : 0;
                const uint64_t dS0 = dil3(S0, S1, S2), dS1 = dil3(S1, S2, S3), dS2 = dil3(S2, S3, S4),
                               dS3 = dil3(S3, S4, S5);
                const uint64_t q0 = t == 0 ? dS0 : ~P0, q1 = t == 0 ? dS1 : ~P1, q2 = t == 0 ? dS2 : ~P2,
                               q3 = t == 0 ? dS3 : ~P3;
                const uint64_t w0 = t == 1 ? S1 : ~S1, w1 = t == 1 ? S2 : ~S2, w2 = t == 1 ? S3 : ~S3,
                               w3 = t == 1 ? S4 : ~S4;
                C0 = w0 & q0 & v0; C1 = w1 & q1 & v1; C2 = w2 & q2 & v2; C3 = w3 & q3 & v3;
                E = (t == 2 && nr == 4) ? (C0 & C1 & C2 & C3 & ~dil3(S0 | S1, S2 | S3, S4 | S5)) : 0ull;
                fresh = 0; x = 0; r = 0; ph = PH_FIND; colx = 0xffffffffu;
            }
            // uniform part: stage the next ring bytes, prefetch every lane's next stripe
            q.sbase = q.fill;
            stage_load(q);
            q.nb4 = ring_get4(Ls.ring, lane, q.bp);
            uint32_t k2 = k, t2 = t, s2 = s, p2 = pidx;
            next_pos3(k2, t2, s2, p2, ns);
            const bool pf = !done && p2 < npasses && k2 < numbps;
            load_rows(X, WS, WS + (WS_BITS + (size_t)(pf ? k2 : 0) * 64) * 64, lane, pf ? 4 * s2 : 0);
        }
        // ---------------- one decision per active lane
        const bool act = !done && !parked;
        step_refill(L, Ls.ring, lane);
        const bool finding = ph == PH_FIND;
        bool pend = act;
        {   // branch-free: every lane runs the search, only finding lanes take its result
            uint32_t fx = x, fr = r;
            const bool found = find_next(C0, C1, C2, C3, fx, fr);
            const bool use = act && finding;
            x = use ? fx : x; r = use ? fr : r;
            pend = use ? found : act;
            parked = parked || (use && !found);
        }
        const uint32_t xc = x & 63;
        const bool is_cl = t == 2, is_mr = t == 1, is_sp = t == 0;
        const bool agg = is_cl && finding && x != colx && ((E >> xc) & 1) && !(xc && ((fresh >> (xc - 1)) & 1));
        colx = (is_cl && finding) ? x : colx;
        const uint32_t sh = 3 * r;
        const uint32_t fs = (win18(S0, S1, S2, S3, S4, S5, xc) >> sh) & 0x1ff;
        const uint32_t fn = (win18(N0, N1, N2, N3, N4, N5, xc) >> sh) & 0x1ff;
        const uint32_t sce = Ls.sc[sc_from9(fs, fn)];
        const uint64_t mu = rsel(r, 0, M0) | rsel(r, 1, M1) | rsel(r, 2, M2) | rsel(r, 3, M3);
        const uint32_t cx_mr = ((mu >> xc) & 1) ? CTX_MAG + 2 : ((fs & 0x1ef) ? CTX_MAG + 1 : CTX_MAG);
        const uint32_t cx = is_mr ? cx_mr
                                  : (agg ? CTX_AGG
                                         : (ph == PH_SIGN ? CTX_SC + (sce & 15)
                                                          : (finding ? CTX_ZC + zc[fs] : CTX_UNI)));
        const uint32_t d = mq_decode(q, L.cw, Ls.tab, cx, pend);
        L.nsym += pend ? 1 : 0;
        // a decoded sign makes the sample significant (SP / CL)
        const bool sig = pend && !is_mr && ph == PH_SIGN;
        const uint64_t bx = sig ? (1ull << xc) : 0ull;
        const uint64_t m0 = rsel(r, 0, bx), m1 = rsel(r, 1, bx), m2 = rsel(r, 2, bx), m3 = rsel(r, 3, bx);
        S1 |= m0; S2 |= m1; S3 |= m2; S4 |= m3;
        const uint64_t ng = (d ^ (sce >> 4)) ? ~0ull : 0ull;
        N1 |= m0 & ng; N2 |= m1 & ng; N3 |= m2 & ng; N4 |= m3 & ng;
        fresh |= bx;
        // plane bit: new significance, or a refinement bit of 1
        const uint64_t pb = bx | ((pend && is_mr && d) ? (1ull << xc) : 0ull);
        B0 |= rsel(r, 0, pb); B1 |= rsel(r, 1, pb); B2 |= rsel(r, 2, pb); B3 |= rsel(r, 3, pb);
        {   // SP: later positions gaining a significant neighbour join the candidates
            const uint64_t bn = is_sp ? bx << 1 : 0ull;
            const uint64_t b0 = rsel(r, 0, bn), b1 = rsel(r, 1, bn), b2 = rsel(r, 2, bn), b3 = rsel(r, 3, bn);
            const uint64_t v0 = nr > 0 ? colmask : 0, v1 = nr > 1 ? colmask : 0, v2 = nr > 2 ? colmask : 0,
                           v3 = nr > 3 ? colmask : 0;
            const uint64_t sp = is_sp ? ~0ull : 0ull;
            C0 |= (b0 | b1) & ~S1 & v0;
            C1 |= ((m0 & sp) | b0 | b1 | b2) & ~S2 & v1;
            C2 |= ((m1 & sp) | b1 | b2 | b3) & ~S3 & v2;
            C3 |= ((m2 & sp) | b2 | b3) & ~S4 & v3;
        }
        // position / phase advance (SP and CL share the CL machine without run-length)
        // (selects, no branches: MR always advances; CL/SP run the phase machine)
        const bool uni1 = ph == PH_UNI1, uni2 = ph == PH_UNI2, sgn = ph == PH_SIGN;
        const bool col_done = !is_mr && agg && !d;
        uint32_t nph = is_mr ? ph
                             : (agg ? (d ? PH_UNI1 : PH_FIND)
                                    : (finding ? (d ? PH_SIGN : PH_FIND) : (uni1 ? PH_UNI2 : (uni2 ? PH_SIGN : PH_FIND))));
        uint32_t nr2 = is_mr ? r + 1
                             : (agg ? r : (finding ? (d ? r : r + 1) : (uni1 ? r : (uni2 ? ((rlhi << 1) | d) : r + 1))));
        (void)sgn;
        rlhi = (pend && !is_mr && uni1) ? d : rlhi;
        nph = pend ? nph : ph;
        nr2 = pend ? (col_done ? 0u : nr2) : r;
        x += (pend && (col_done || nr2 == 4)) ? 1 : 0;
        ph = nph;
        r = nr2 & 3;
        step_prefetch(L, Ls.ring, lane);
    }
    if (stats) {
        unsigned long long tot = L.nsym;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        if (lane == 0) atomicAdd(&stats[3], (unsigned long long)nevents);
        if (lane == 0) { atomicAdd(&stats[0], (unsigned long long)L.step); atomicAdd(&stats[1], tot);
                         atomicMax(&stats[2], (unsigned long long)L.step); }
    }
}

// =============================================================================
// Variant 2 (default): lane-independent stepping with the stripe state in LDS.
//
// Measured on variant 1 (SQ counters, C2): one wave per SIMD spends 72 % of its
// cycles issuing ~600 instructions per decision, so the kernel is bound by the
// instruction count of one step (a wave alone issues one VALU per 4 cycles).
// This variant cuts the step to what the decision needs:
//  * the stripe's significance and sign rows live in LDS, per lane, in a
//    guarded layout (bit c+1 = column c, three dwords per row, [dword][lane]),
//    so the 3x3 neighbourhood of (x, r) is three ds_read2st64 + alignbit, and a
//    new significance is one ds_or_b32 - no per-row register selects;
//  * refinement (mu) and plane-bit rows live in LDS too (read / or per step);
//  * candidates are consumed: the next coding position is the first set bit of
//    the candidate rows (one col4 per step); propagation in SP follows from the
//    neighbourhood window already read;
//  * the MQ code register is a 64-bit bit buffer (Chigh at bits 63:48, code
//    bits pre-loaded below it, one byte inserted per step), so RENORMD is one
//    shift with no byte loop (Annex C.3.3 / C.3.4 restated).
// Stripe boundaries (batched, as in variant 1) move rows between scratch,
// registers and LDS.
// =============================================================================
struct Mq2 {
    uint64_t c;                  // bits 63:48 = Chigh; `avail` valid code bits below bit 48
    uint32_t a, avail;
    uint32_t bp, len, fill;      // byte position (last byte taken in), block length, ring fill position
    uint32_t nb4;                // bytes [bp, bp + 4)
    uint32_t sbase;              // staged bytes cover [sbase, sbase + 32)
    uint32_t T0, T1, T2, T3, T4, T5, T6, T7;
    const uint8_t* p;
};

// BYTEIN ahead of need (mqc_dec.cpp BYTEIN, Annex C.3.4): the byte after the last one taken
// goes below the valid bits; after 0xFF it overlaps by one bit (B << 9), a marker feeds 1s.
__device__ __forceinline__ void mq2_refill(Mq2& q, bool en) {
    const uint32_t cur = q.nb4 & 0xff, nxt = (q.nb4 >> 8) & 0xff;   // ring bytes past the end are 0xFF
    const bool ff = cur == 0xff, stuck = ff & (nxt > 0x8f);
    const bool seven = ff & !stuck;
    const uint32_t add = en ? (stuck ? 0xffu : nxt) : 0u;
    const uint32_t sh = (40u + (seven ? 1u : 0u) - q.avail) & 63;
    q.c += (uint64_t)add << sh;
    q.avail += en ? (seven ? 7u : 8u) : 0u;
    const bool adv = en && !stuck;
    q.bp += adv ? 1u : 0u;
    q.nb4 = adv ? (q.nb4 >> 8) : q.nb4;
}

// DECODE (Annex C.3.2) for context cx, predicated on `en`; needs avail >= 15.
__device__ __forceinline__ uint32_t mq2_decode(Mq2& q, Ctx5& cw, const uint32_t* tab, uint32_t cx, bool en) {
    const uint32_t wi = cx >> 2, shb = (cx & 3) * 8;
    uint32_t word = vsel(wi == 4, cw.w4, vsel(wi & 2, vsel(wi & 1, cw.w3, cw.w2), vsel(wi & 1, cw.w1, cw.w0)));
    const uint32_t st = (word >> shb) & 0xff;
    const uint32_t mps = st >> 6;
    const uint32_t e = tab[st & 63];
    const uint32_t qe = e & 0xffff;
    const uint32_t chi = (uint32_t)(q.c >> 32);
    const uint32_t a1 = q.a - qe;
    const bool lower = (chi >> 16) < qe;
    const bool fast = !lower && (a1 & 0x8000);
    const bool mps_path = lower ? (a1 < qe) : (a1 >= qe);
    const uint32_t d = (fast || mps_path) ? mps : (mps ^ 1);
    const uint32_t nst = mps_path ? (((e >> 16) & 0x3f) | (mps << 6)) : (((e >> 22) & 0x3f) | ((mps ^ (e >> 28)) << 6));
    const bool upd = en && !fast;
    const uint32_t an = en ? (lower ? qe : a1) : q.a;
    const uint32_t ch = (en && !lower) ? chi - (qe << 16) : chi;
    word = (word & ~(0xffu << shb)) | (nst << shb);
    const uint32_t wu = upd ? wi : 7u;
    cw.w0 = vsel(wu == 0, word, cw.w0); cw.w1 = vsel(wu == 1, word, cw.w1);
    cw.w2 = vsel(wu == 2, word, cw.w2); cw.w3 = vsel(wu == 3, word, cw.w3);
    cw.w4 = vsel(wu == 4, word, cw.w4);
    const uint32_t n = upd ? __clz(an) - 16 : 0u;   // RENORMD: all shifts at once
    q.a = an << n;
    q.c = (((uint64_t)ch << 32) | (uint32_t)q.c) << n;
    q.avail -= n;
    return d;
}

struct Dec2Lds {
    uint32_t tab[48];
    uint8_t zc[4][512];
    uint8_t sc[256];                 // index bit0 N-neg 1 N-sig 2 W-neg 3 W-sig 4 E-neg 5 E-sig 6 S-neg 7 S-sig
    uint32_t ring[RING_DW + 1][64];
    uint32_t sg[6 * 3][64];          // significance rows y0-1 .. y0+4, guarded: bit c+1 of the 96-bit row = column c
    uint32_t ng[6 * 3][64];          // sign rows (bits only where significant), same layout
    uint32_t mu[4 * 2][64];          // refined-in-an-earlier-plane rows y0 .. y0+3, plain 32-bit halves
    uint32_t bt[4 * 2][64];          // plane-bit rows y0 .. y0+3
};

__device__ __forceinline__ void g_put(uint32_t (*g)[64], int row, int lane, uint64_t v) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    g[row * 3][lane] = lo << 1;
    g[row * 3 + 1][lane] = __builtin_amdgcn_alignbit(hi, lo, 31);
    g[row * 3 + 2][lane] = hi >> 31;
}
__device__ __forceinline__ uint64_t g_get(uint32_t (*g)[64], int row, int lane) {
    const uint32_t d0 = g[row * 3][lane], d1 = g[row * 3 + 1][lane], d2 = g[row * 3 + 2][lane];
    return ((uint64_t)__builtin_amdgcn_alignbit(d2, d1, 1) << 32) | __builtin_amdgcn_alignbit(d1, d0, 1);
}
__device__ __forceinline__ void h_put(uint32_t (*g)[64], int row, int lane, uint64_t v) {
    g[row * 2][lane] = (uint32_t)v;
    g[row * 2 + 1][lane] = (uint32_t)(v >> 32);
}
__device__ __forceinline__ uint64_t h_get(uint32_t (*g)[64], int row, int lane) {
    return ((uint64_t)g[row * 2 + 1][lane] << 32) | g[row * 2][lane];
}

// TIMING (diagnostic build, GK_T1_STATS=2): shader-clock cycles spent in stripe-boundary
// events vs decision steps, summed into stats[4] / stats[5].
template <bool TIMING>
__global__ __launch_bounds__(64) void k_t1_dec2(const uint8_t* __restrict__ bytes, const GkBlock* __restrict__ blocks,
                                                const uint32_t* __restrict__ order, uint64_t* __restrict__ scratch,
                                                const uint64_t* __restrict__ wave_off, uint32_t nblocks,
                                                unsigned long long* __restrict__ stats, uint32_t kpark) {
    __shared__ Dec2Lds Ls;
    const int lane = threadIdx.x;
    if (lane < 47) Ls.tab[lane] = c_mq[lane];
    for (int i = lane; i < 2048; i += 64) Ls.zc[i >> 9][i & 511] = zc_rule((uint32_t)(i >> 9), (uint32_t)(i & 511));
    for (int i = lane; i < 256; i += 64)
        Ls.sc[i] = sc_rule((uint32_t)(((i >> 2) & 0xf) | ((i & 3) << 4) | (i & 0xc0)));
    const uint32_t slot = blockIdx.x * 64 + lane;
    const uint32_t bid = slot < nblocks ? order[slot] : 0xffffffffu;   // empty slots: 0xffffffff
    const bool has = bid != 0xffffffffu;
    GkBlock B = {};
    if (has) B = blocks[bid];
    uint64_t* WS = scratch + wave_off[blockIdx.x];
    const uint32_t numbps = has ? B.numbps : 0, npasses = (has && B.numbps) ? B.npasses : 0;
    const uint32_t h = B.h, w = B.w;
    const uint64_t colmask = w >= 64 ? ~0ull : ((1ull << w) - 1);
    const uint32_t ns = (h + 3) >> 2;
    const uint8_t* zc = Ls.zc[B.orient & 3];
    for (int r = 0; r < WS_FIXED; ++r) WS[r * 64 + lane] = 0;   // clear the state rows (coalesced)
    for (int i = 0; i < 18; ++i) { Ls.sg[i][lane] = 0; Ls.ng[i][lane] = 0; }
    for (int i = 0; i < 8; ++i) { Ls.mu[i][lane] = 0; Ls.bt[i][lane] = 0; }
    Ctx5 cw = {4u, 0u, 0u, 0u, (3u << 8) | (46u << 16)};   // mqc_resetstates: ZC0=4, AGG=3, UNI=46
    uint32_t nstep = 0, nsym = 0, nevents = 0;
    unsigned long long cyc_ev = 0, cyc_step = 0;
    Mq2 q;
    q.p = npasses ? bytes + B.data_off : bytes;
    q.len = npasses ? B.len : 0;
    q.bp = 0; q.fill = 0; q.sbase = 0;
    stage_load(q);
    __syncthreads();
    ring_boundary(Ls.ring, lane, q);
    ring_boundary(Ls.ring, lane, q);
    ring_boundary(Ls.ring, lane, q);
    // INITDEC (mqc_dec.cpp:98-112): C = B0 << 16, BYTEIN, C <<= 7, CT -= 7, A = 0x8000
    q.nb4 = ring_get4(Ls.ring, lane, 0);
    q.c = (uint64_t)(q.len ? (q.nb4 & 0xff) : 0xffu) << 48;
    q.avail = 0;
    mq2_refill(q, true);
    q.c <<= 7; q.avail -= 7; q.a = 0x8000;
#pragma unroll
    for (int i = 0; i < 5; ++i) { q.nb4 = ring_get4(Ls.ring, lane, q.bp); mq2_refill(q, q.avail <= 40); }
    q.nb4 = ring_get4(Ls.ring, lane, q.bp);

    // position: plane k (0 = top), pass type t (0 SP, 1 MR, 2 CL), stripe s, pass index pidx
    uint32_t k = 0, t = 2, s = 0, pidx = 0;
    bool done = npasses == 0, parked = false;
    uint32_t nr = min(4u, h), x = 0, r = 0, ph = PH_FIND, rlhi = 0;
    uint32_t vr = (1u << nr) - 1;                 // valid rows of the stripe
    uint64_t C0, C1, C2, C3, E, fresh = 0;        // candidates (consumed as coded), run-length columns
    uint64_t P0 = 0, P1 = 0, P2 = 0, P3 = 0;      // visited in SP of this plane
    uint64_t M0 = 0, M1 = 0, M2 = 0, M3 = 0;      // refined rows after this stripe-pass
    {
        const uint64_t v0 = nr > 0 ? colmask : 0, v1 = nr > 1 ? colmask : 0, v2 = nr > 2 ? colmask : 0,
                       v3 = nr > 3 ? colmask : 0;
        C0 = v0; C1 = v1; C2 = v2; C3 = v3;      // first CL: nothing significant yet
        E = (nr == 4) ? colmask : 0ull;
    }
    Rows22 X = {};
    {
        uint32_t k2 = k, t2 = t, s2 = s, p2 = pidx;
        next_pos3(k2, t2, s2, p2, ns);
        if (!done && p2 < npasses && k2 < numbps) load_rows(X, WS, WS + (WS_BITS + (size_t)k2 * 64) * 64, lane, 4 * s2);
    }

    while (__any(!done)) {
        // ---------------- stripe boundary for parked lanes (batched)
        const uint32_t nparked = __popcll(__ballot(parked));
        const uint32_t nactive = __popcll(__ballot(!done && !parked));
        uint64_t tev = 0;
        if (nparked && (nparked >= kpark || nactive == 0)) {
            ++nevents;
            if (TIMING) tev = __builtin_amdgcn_s_memtime();
            if (!done && q.sbase == q.fill && q.fill + 32 - q.bp <= 4 * RING_DW) {
                ring_write16(Ls.ring, lane, q.fill, q.T0, q.T1, q.T2, q.T3, q.len);
                ring_write16(Ls.ring, lane, q.fill + 16, q.T4, q.T5, q.T6, q.T7, q.len);
                q.fill += 32;
            }
            if (parked) {
                parked = false;
                const uint32_t y0 = 4 * s;
                // the finished stripe: rows back to scratch
                const uint64_t S1 = g_get(Ls.sg, 1, lane), S2 = g_get(Ls.sg, 2, lane), S3 = g_get(Ls.sg, 3, lane),
                               S4 = g_get(Ls.sg, 4, lane);
                const uint64_t N1 = g_get(Ls.ng, 1, lane), N2 = g_get(Ls.ng, 2, lane), N3 = g_get(Ls.ng, 3, lane),
                               N4 = g_get(Ls.ng, 4, lane);
                const uint64_t B0 = h_get(Ls.bt, 0, lane), B1 = h_get(Ls.bt, 1, lane), B2 = h_get(Ls.bt, 2, lane),
                               B3 = h_get(Ls.bt, 3, lane);
                uint64_t* sgp = WS + (size_t)(WS_SIG + y0 + 1) * 64 + lane;
                uint64_t* ngp = WS + (size_t)(WS_NEG + y0 + 1) * 64 + lane;
                uint64_t* pip = WS + (size_t)(WS_PI + y0) * 64 + lane;
                uint64_t* btp = WS + (WS_BITS + (size_t)k * 64 + y0) * 64 + lane;
                sgp[0] = S1; sgp[64] = S2; sgp[128] = S3; sgp[192] = S4;
                ngp[0] = N1; ngp[64] = N2; ngp[128] = N3; ngp[192] = N4;
                if (t == 0) { pip[0] = P0; pip[64] = P1; pip[128] = P2; pip[192] = P3; }
                btp[0] = B0; btp[64] = B1; btp[128] = B2; btp[192] = B3;
                const uint32_t ok = k;
                next_pos3(k, t, s, pidx, ns);
                done = pidx >= npasses || k >= numbps;
                // new stripe rows: prefetched, except rows the finished stripe still held when the
                // prefetch was issued (1-stripe blocks: all; 2-stripe blocks at a pass change: row 4)
                const bool one = ns == 1, two = ns == 2 && s == 0;
                const uint64_t nS0 = s ? S4 : 0ull, nN0 = s ? N4 : 0ull;
                const uint64_t nS1 = one ? S1 : X.s1, nS2 = one ? S2 : X.s2, nS3 = one ? S3 : X.s3, nS4 = one ? S4 : X.s4;
                const uint64_t nS5 = two ? S1 : X.s5;
                const uint64_t nN1 = one ? N1 : X.n1, nN2 = one ? N2 : X.n2, nN3 = one ? N3 : X.n3, nN4 = one ? N4 : X.n4;
                const uint64_t nN5 = two ? N1 : X.n5;
                const uint64_t nP0 = one ? P0 : X.p0, nP1 = one ? P1 : X.p1, nP2 = one ? P2 : X.p2, nP3 = one ? P3 : X.p3;
                const uint64_t nM0 = one ? M0 : X.m0, nM1 = one ? M1 : X.m1, nM2 = one ? M2 : X.m2, nM3 = one ? M3 : X.m3;
                const bool same_plane = one && ok == k;
                const bool newplane = t == 0 || k == 0;
                const uint64_t nB0 = newplane ? 0ull : (same_plane ? B0 : X.b0), nB1 = newplane ? 0ull : (same_plane ? B1 : X.b1),
                               nB2 = newplane ? 0ull : (same_plane ? B2 : X.b2), nB3 = newplane ? 0ull : (same_plane ? B3 : X.b3);
                const uint64_t pP0 = t == 0 ? 0ull : nP0, pP1 = t == 0 ? 0ull : nP1, pP2 = t == 0 ? 0ull : nP2,
                               pP3 = t == 0 ? 0ull : nP3;
                g_put(Ls.sg, 0, lane, nS0); g_put(Ls.sg, 1, lane, nS1); g_put(Ls.sg, 2, lane, nS2);
                g_put(Ls.sg, 3, lane, nS3); g_put(Ls.sg, 4, lane, nS4); g_put(Ls.sg, 5, lane, nS5);
                g_put(Ls.ng, 0, lane, nN0); g_put(Ls.ng, 1, lane, nN1); g_put(Ls.ng, 2, lane, nN2);
                g_put(Ls.ng, 3, lane, nN3); g_put(Ls.ng, 4, lane, nN4); g_put(Ls.ng, 5, lane, nN5);
                h_put(Ls.mu, 0, lane, nM0); h_put(Ls.mu, 1, lane, nM1); h_put(Ls.mu, 2, lane, nM2); h_put(Ls.mu, 3, lane, nM3);
                h_put(Ls.bt, 0, lane, nB0); h_put(Ls.bt, 1, lane, nB1); h_put(Ls.bt, 2, lane, nB2); h_put(Ls.bt, 3, lane, nB3);
                const uint32_t ny0 = 4 * s;
                nr = done ? 0u : min(4u, h - ny0);
                vr = (1u << nr) - 1;
                const uint64_t v0 = nr > 0 ? colmask : 0, v1 = nr > 1 ? colmask : 0, v2 = nr > 2 ? colmask : 0,
                               v3 = nr > 3 ? colmask : 0;
                const uint64_t dS0 = dil3(nS0, nS1, nS2), dS1 = dil3(nS1, nS2, nS3), dS2 = dil3(nS2, nS3, nS4),
                               dS3 = dil3(nS3, nS4, nS5);
                const uint64_t q0 = t == 0 ? dS0 : ~pP0, q1 = t == 0 ? dS1 : ~pP1, q2 = t == 0 ? dS2 : ~pP2,
                               q3 = t == 0 ? dS3 : ~pP3;
                const uint64_t w0 = t == 1 ? nS1 : ~nS1, w1 = t == 1 ? nS2 : ~nS2, w2 = t == 1 ? nS3 : ~nS3,
                               w3 = t == 1 ? nS4 : ~nS4;
                C0 = w0 & q0 & v0; C1 = w1 & q1 & v1; C2 = w2 & q2 & v2; C3 = w3 & q3 & v3;
                E = (t == 2 && nr == 4) ? (C0 & C1 & C2 & C3 & ~dil3(nS0 | nS1, nS2 | nS3, nS4 | nS5)) : 0ull;
                // SP: visited = its candidates (grown by propagation); MR: refined = old | coded now
                P0 = t == 0 ? C0 : pP0; P1 = t == 0 ? C1 : pP1; P2 = t == 0 ? C2 : pP2; P3 = t == 0 ? C3 : pP3;
                M0 = nM0 | (t == 1 ? C0 : 0ull); M1 = nM1 | (t == 1 ? C1 : 0ull);
                M2 = nM2 | (t == 1 ? C2 : 0ull); M3 = nM3 | (t == 1 ? C3 : 0ull);
                if (t == 1) {
                    uint64_t* mup = WS + (size_t)(WS_MU + ny0) * 64 + lane;
                    mup[0] = M0; mup[64] = M1; mup[128] = M2; mup[192] = M3;
                }
                fresh = 0; ph = PH_FIND;
            }
            q.sbase = q.fill;
            stage_load(q);
            uint32_t k2 = k, t2 = t, s2 = s, p2 = pidx;
            next_pos3(k2, t2, s2, p2, ns);
            const bool pf = !done && p2 < npasses && k2 < numbps;
            load_rows(X, WS, WS + (WS_BITS + (size_t)(pf ? k2 : 0) * 64) * 64, lane, pf ? 4 * s2 : 0);
            if (TIMING) { const uint64_t t1 = __builtin_amdgcn_s_memtime(); cyc_ev += t1 - tev; tev = t1; }
        }
        if (TIMING && !tev) tev = __builtin_amdgcn_s_memtime();
        // ---------------- one decision per active lane
        const bool act = !done && !parked;
        ++nstep;
        if (__any(q.fill - q.bp < 8)) ring_topup(Ls.ring, lane, q);
        mq2_refill(q, act && q.avail <= 40);
        const bool finding = ph == PH_FIND;
        // next coding position: first remaining candidate in stripe scan order
        const uint64_t CU = C0 | C1 | C2 | C3;
        const uint32_t xq = ((uint32_t)__ffsll((long long)CU) - 1) & 63;
        const uint32_t c4 = col4(C0, C1, C2, C3, xq);
        const bool use = act && finding;
        const bool found = CU != 0;
        x = (use && found) ? xq : x;
        r = (use && found) ? (uint32_t)(__ffs(c4) - 1) : r;
        const bool pend = use ? found : act;
        parked = parked || (use && !found);
        // neighbourhood of (x, r): guarded rows r .. r+2 (= stripe rows r-1 .. r+1)
        const uint32_t dx = x >> 5, sx = x & 31;
        const uint32_t o0 = (r * 3 + dx);
        const uint32_t s0 = __builtin_amdgcn_alignbit(Ls.sg[o0 + 1][lane], Ls.sg[o0][lane], sx) & 7;
        const uint32_t s1 = __builtin_amdgcn_alignbit(Ls.sg[o0 + 4][lane], Ls.sg[o0 + 3][lane], sx) & 7;
        const uint32_t s2 = __builtin_amdgcn_alignbit(Ls.sg[o0 + 7][lane], Ls.sg[o0 + 6][lane], sx) & 7;
        const uint32_t n0 = __builtin_amdgcn_alignbit(Ls.ng[o0 + 1][lane], Ls.ng[o0][lane], sx) & 7;
        const uint32_t n1 = __builtin_amdgcn_alignbit(Ls.ng[o0 + 4][lane], Ls.ng[o0 + 3][lane], sx) & 7;
        const uint32_t n2 = __builtin_amdgcn_alignbit(Ls.ng[o0 + 7][lane], Ls.ng[o0 + 6][lane], sx) & 7;
        const uint32_t mub = (Ls.mu[r * 2 + dx][lane] >> sx) & 1;
        const uint32_t fs = s0 | (s1 << 3) | (s2 << 6);
        const uint32_t fn = n0 | (n1 << 3) | (n2 << 6);
        const uint32_t sce = Ls.sc[(fs & 0xaa) | ((fn >> 1) & 0x55)];
        const uint32_t zcx = zc[fs];
        const bool is_cl = t == 2, is_mr = t == 1, is_sp = t == 0;
        // a column starts in run-length mode when it was eligible at stripe start, is untouched
        // and its left neighbour column gained no significance in this pass
        // (bitwise, not short-circuit: keeps the step free of exec-mask branches)
        const bool agg = is_cl & finding & (((E >> x) & 1) != 0) & (c4 == 0xf) & ((((fresh << 1) >> x) & 1) == 0);
        const uint32_t cx_mr = vsel(mub != 0, CTX_MAG + 2, vsel((fs & 0x1ef) != 0, CTX_MAG + 1, CTX_MAG));
        const uint32_t cx = vsel(is_mr, cx_mr,
                                 vsel(agg, CTX_AGG,
                                      vsel(ph == PH_SIGN, CTX_SC + (sce & 15), vsel(finding, CTX_ZC + zcx, CTX_UNI))));
        while (__any(pend && q.avail < 16)) {   // rare: a burst of long renormalisations
            mq2_refill(q, pend && q.avail < 16);
            q.nb4 = ring_get4(Ls.ring, lane, q.bp);
        }
        const uint32_t d = mq2_decode(q, cw, Ls.tab, cx, pend);
        nsym += pend ? 1 : 0;
        // ---- state updates
        const bool sig = pend && !is_mr && ph == PH_SIGN;
        const bool negs = sig && ((d ^ (sce >> 4)) & 1);
        const uint32_t gx = x + 1, gd = gx >> 5, gb = 1u << (gx & 31);
        atomicOr(&Ls.sg[(r + 1) * 3 + gd][lane], sig ? gb : 0u);
        atomicOr(&Ls.ng[(r + 1) * 3 + gd][lane], negs ? gb : 0u);
        const bool pb = sig || (pend && is_mr && d);
        atomicOr(&Ls.bt[r * 2 + dx][lane], pb ? (1u << sx) : 0u);
        fresh |= (uint64_t)(sig ? 1u : 0u) << x;
        // SP: positions after (x, r) that gain a significant neighbour become candidates:
        // (x, r+1) and column x+1 rows r-1 .. r+1, unless significant (window bits 7; 2, 5, 8)
        const bool spn = sig && is_sp;
        const uint32_t nf = ~fs;
        const uint32_t ca = spn ? ((((nf >> 7) & 1) << (r + 1)) & vr) : 0u;
        const uint32_t t3 = ((nf >> 2) & 1) | ((nf >> 4) & 2) | ((nf >> 6) & 4);
        const uint32_t cb = (spn && gx < w) ? (((t3 << r) >> 1) & vr) : 0u;
        // consumption: the coded position; a whole column after a zero run-length decision;
        // rows 0 .. rr once the run-length index rr is known
        const uint32_t rr = (rlhi << 1) | d;
        const uint32_t crow_f = vsel(agg, vsel(d != 0, 0u, 0xfu), 1u << r);
        const uint32_t crow = vsel(pend, vsel(finding, crow_f, vsel(ph == PH_UNI2, (2u << rr) - 1, 0u)), 0u);
#define GK_CROW(Ci, Pi, i)                                                                                           \
    {                                                                                                                \
        const uint64_t add = (uint64_t)(((ca >> i) & 1) | (((cb >> i) & 1) << 1)) << x;                             \
        const uint64_t clr = (uint64_t)((crow >> i) & 1) << x;                                                       \
        Ci = (Ci & ~clr) | add;                                                                                      \
        Pi |= add;                                                                                                   \
    }
        GK_CROW(C0, P0, 0) GK_CROW(C1, P1, 1) GK_CROW(C2, P2, 2) GK_CROW(C3, P3, 3)
#undef GK_CROW
        // phase machine: FIND -(ZC 1)-> SIGN -> FIND; FIND(run-length) -(1)-> UNI1 -> UNI2 -> SIGN
        // next phase = table[ph][d][agg] (MR always stays in FIND), 2 bits per entry
        //   FIND: agg ? (d ? UNI1 : FIND) : (d ? SIGN : FIND); SIGN -> FIND; UNI1 -> UNI2; UNI2 -> SIGN
        const bool uni1 = ph == PH_UNI1, uni2 = ph == PH_UNI2;
        const uint32_t key = (ph << 2) | (d << 1) | (agg ? 1u : 0u);
        constexpr uint32_t kPhT = (0u << 0) | (0u << 2) | (PH_SIGN << 4) | (PH_UNI1 << 6)       // FIND
                                | (PH_UNI2 << 16) | (PH_UNI2 << 18) | (PH_UNI2 << 20) | (PH_UNI2 << 22)  // UNI1
                                | (PH_SIGN << 24) | (PH_SIGN << 26) | (PH_SIGN << 28) | (PH_SIGN << 30); // UNI2
        const uint32_t nph = is_mr ? (uint32_t)PH_FIND : ((kPhT >> (2 * key)) & 3);
        rlhi = vsel(pend & uni1, d, rlhi);
        r = vsel(pend & uni2, rr, r);
        ph = vsel(pend, nph, ph);
        q.nb4 = ring_get4(Ls.ring, lane, q.bp);
        if (TIMING) cyc_step += __builtin_amdgcn_s_memtime() - tev;
    }
    if (stats) {
        unsigned long long tot = nsym;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        if (lane == 0) {
            if (TIMING) { atomicAdd(&stats[4], cyc_ev); atomicAdd(&stats[5], cyc_step); }
            atomicAdd(&stats[3], (unsigned long long)nevents);
            atomicAdd(&stats[0], (unsigned long long)nstep); atomicAdd(&stats[1], tot);
            atomicMax(&stats[2], (unsigned long long)nstep);
        }
    }
}

// Reconstruction + dequantisation: wave per block, lane = column.
// Job q reconstructs block ids[q], whose decoder lane was pos[q].
__global__ __launch_bounds__(64) void k_t1_recon(const GkBlock* __restrict__ blocks, const uint32_t* __restrict__ ids,
                                                 const uint32_t* __restrict__ pos,
                                                 const uint64_t* __restrict__ scratch,
                                                 const uint64_t* __restrict__ wave_off, int32_t* __restrict__ coef,
                                                 uint32_t nblocks) {
    const uint32_t q = blockIdx.x;
    if (q >= nblocks) return;
    const int x = threadIdx.x;
    const GkBlock B = blocks[ids[q]];
    if (x >= (int)B.w) return;
    const uint32_t slot = pos[q], ln = slot & 63;
    const uint64_t* WS = scratch + wave_off[slot >> 6];
    const bool irrev = B.flags & 1;
    float* fcoef = reinterpret_cast<float*>(coef);
    const uint32_t numbps = B.numbps, npasses = B.npasses;
    // last decoded pass k = npasses-1: pass k>0 belongs to plane numbps-1-(k+2)/3, type (k+2)%3
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
                uint64_t row = WS[(WS_BITS + (size_t)(numbps - 1 - p) * 64 + y) * 64 + ln];
                M |= (uint32_t)((row >> x) & 1) << p;
            }
            if (M) {
                int qq = (t == 0 && (M >> (bpl + 1)) != 0) ? bpl + 1 : bpl;
                int32_t mag = (int32_t)(((M >> qq) << 1 | 1) << qq);
                bool ng = (WS[(WS_NEG + y + 1) * 64 + ln] >> x) & 1;
                v = ng ? -mag : mag;
            }
        }
        size_t o = B.band_off + (size_t)y * B.stride + x;
        if (irrev) fcoef[o] = (float)v * B.step;
        else coef[o] = v / 2;
    }
}

#include "gk_launch.h"
// Blocks per 64-lane wave (GK_T1DEC_LANES, 1..64).
uint32_t gk_t1dec_lanes() {
    static uint32_t lanes = 0;
    if (!lanes) {
        const char* v = getenv("GK_T1DEC_LANES");
        int n = v ? atoi(v) : 64;
        lanes = (uint32_t)(n < 1 ? 1 : (n > 64 ? 64 : n));
    }
    return lanes;
}
void gk_launch_t1_dec(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, const uint32_t* order,
                      uint64_t* scratch, const uint64_t* wave_off, uint32_t nblocks) {
    if (!nblocks) return;
    static unsigned long long* stats = nullptr;
    const char* sv = getenv("GK_T1_STATS");
    const bool want = sv != nullptr, timing = sv && atoi(sv) == 2;
    if (want && !stats) { (void)hipMalloc(&stats, 64); }
    if (want) (void)hipMemsetAsync(stats, 0, 64, st);
    static int variant = -1, kpark = 4;
    if (variant < 0) {
        const char* v = getenv("GK_T1DEC");   // 0: stripe-synchronous, 1: lane-independent, 2 (default): LDS state
        variant = v ? atoi(v) : 2;
        const char* kp = getenv("GK_T1DEC_PARK");
        if (kp) kpark = atoi(kp);
    }
    if (variant == 0)
        hipLaunchKernelGGL(k_t1_dec, dim3((nblocks + 63) / 64), dim3(64), 0, st, bytes, blocks, order, scratch,
                           wave_off, nblocks, want ? stats : nullptr);
    else if (variant == 2 && timing)
        hipLaunchKernelGGL(k_t1_dec2<true>, dim3((nblocks + 63) / 64), dim3(64), 0, st, bytes, blocks, order, scratch,
                           wave_off, nblocks, stats, (uint32_t)kpark);
    else if (variant == 2)
        hipLaunchKernelGGL(k_t1_dec2<false>, dim3((nblocks + 63) / 64), dim3(64), 0, st, bytes, blocks, order, scratch,
                           wave_off, nblocks, want ? stats : nullptr, (uint32_t)kpark);
    else
        hipLaunchKernelGGL(k_t1_dec_ind, dim3((nblocks + 63) / 64), dim3(64), 0, st, bytes, blocks, order, scratch,
                           wave_off, nblocks, want ? stats : nullptr, (uint32_t)kpark);
    if (want) {
        unsigned long long h[8];
        (void)hipMemcpyAsync(h, stats, 64, hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
        fprintf(stderr, "t1dec stats: waves %u steps_total %llu symbols %llu max_steps %llu avg_steps/wave %.0f lane_eff %.3f events/wave %.0f\n",
                (nblocks + 63) / 64, h[0], h[1], h[2], (double)h[0] / ((nblocks + 63) / 64), (double)h[1] / (64.0 * h[0]),
                (double)h[3] / ((nblocks + 63) / 64));
        if (timing)
            fprintf(stderr, "t1dec timing: cycles/event %.0f cycles/step %.0f (event share %.3f)\n",
                    (double)h[4] / (double)(h[3] ? h[3] : 1), (double)h[5] / (double)(h[0] ? h[0] : 1),
                    (double)h[4] / (double)(h[4] + h[5] ? h[4] + h[5] : 1));
    }
}
void gk_launch_t1_recon(hipStream_t st, const GkBlock* blocks, const uint32_t* ids, const uint32_t* pos,
                        const uint64_t* scratch, const uint64_t* wave_off, int32_t* coef, uint32_t nblocks) {
    if (!nblocks) return;
    hipLaunchKernelGGL(k_t1_recon, dim3(nblocks), dim3(64), 0, st, blocks, ids, pos, scratch, wave_off, coef, nblocks);
}
