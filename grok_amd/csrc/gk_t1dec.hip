// gk_t1dec.hip — Part-1 T1 decoder for CDNA4: one lane per code-block,
// lane-independent stepping, stripe state in LDS.
//
// Decoding is a serial chain per code-block (every MQ decision feeds the next
// context; T1::decompress_cblk, T1.cpp:934-1446), so the parallelism is the
// code-blocks: each lane of a wave decodes its own block, one MQ decision per
// step.  Every lane walks its own (bit-plane, pass, stripe) sequence; a step
// decodes whatever its lane needs next (SP / MR / CL share one branch-free
// step), so the wave's loop runs as long as its heaviest block, not the sum of
// per-stripe maxima.  Blocks are assigned to lanes sorted by pass count (host),
// so the lanes of a wave carry similar work.
//
// Measured (SQ counters, C2): with one wave per SIMD the kernel is bound by the
// instructions of one step (a wave alone issues a VALU every 4 cycles), so the
// design minimises instructions per decision:
//  * the stripe's significance and sign rows live in LDS, per lane, in a
//    guarded layout (bit c+1 = column c, three dwords per row, [dword][lane]):
//    the 3x3 neighbourhood of (x, r) is three ds_read2st64 + alignbit, and a
//    new significance is one ds_or_b32 - no per-row register selects;
//  * refinement (mu) and plane-bit rows live in LDS too;
//  * candidates are consumed: the next coding position is the first set bit of
//    the candidate rows; SP propagation follows from the neighbourhood window;
//  * the MQ code register is a 64-bit bit buffer (Chigh at bits 63:48, code
//    bits pre-loaded below it, one byte inserted per step), so RENORMD is one
//    shift with no byte loop (Annex C.3.3 / C.3.4 restated).
// A lane whose stripe-pass has no candidate left parks; parked lanes cross their
// stripe boundary together once `kpark` of them wait, moving rows between the
// per-lane scratch (contiguous rows per lane), registers and LDS; the next
// stripe's rows are prefetched at the previous boundary.
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
#include <algorithm>
#include <string>

// per-lane scratch (uint64 words, one contiguous slab per lane, 128-byte aligned).  A stripe's
// state rows are one 128-byte line: stripe s at 16 s holds significance, sign, visited (SP of the
// current plane) and refined-in-an-earlier-plane rows 4s .. 4s+3, four words each, so a stripe
// boundary moves whole lines (plus the first rows of the next stripe's line: the row below).
// Stripe 16 is an all-zero guard.  The decoded bit-plane rows follow, plane-major.
#define WS_S 0        // + 16 s + (y & 3): significance of row y = 4 s + (y & 3)
#define WS_N 4        // sign (set where significant)
#define WS_P 8        // visited in SP of the current plane
#define WS_M 12       // refined in an earlier plane
#define WS_BITS 272   // numbps planes x 64 rows: bit of the plane (plane 0 = most significant)
#define WS_FIXED 272

// ------------------------------------------------------------------ MQ byte ring
// Compressed bytes reach the coder through a 128-byte per-lane ring in LDS
// (dword-interleaved [dword][lane], conflict-free).  Refills happen at stripe
// boundaries: the 32 bytes staged in VGPRs by the previous boundary are written
// and the next 32 are requested, so no step waits on global memory.  A lane whose
// ring runs low inside a dense stripe-pass takes a synchronous top-up (rare).
// At the end of every step each lane reads the 4 bytes at its position (nb4).
#define RING_DW 32
#ifndef T1DEC_UNROLL
#define T1DEC_UNROLL 16   // decision steps per stripe-boundary test (round 2, C2 decoder: 1 -> 33.5 ms, 8 -> 26.4, 12 -> 25.8, 16 -> 26.3; round 4 with solo waves: 10 -> 20.6, 12 -> 20.5, 16 -> 20.3, 20 -> 20.2-20.3, 24 -> 20.4)
#endif
__device__ __forceinline__ uint32_t vsel(bool c, uint32_t a, uint32_t b) {
    // per-lane select; a plain ternary lets the compiler keep c as the compare's lane mask (an
    // explicit ballot made it rebuild the mask from a 0/1 value: two extra instructions each)
    return c ? a : b;
}

// Bytes at or past the block length read as 0xFF (the MQ decoder's end-of-data rule,
// mqc_dec.cpp BYTEIN).  The host pads every staged block with >= 32 bytes of 0xFF after its
// data, and windows that start at or past the length read this constant instead, so the
// ring needs no per-byte length tests.
__device__ uint4 g_ff32[2] = {{~0u, ~0u, ~0u, ~0u}, {~0u, ~0u, ~0u, ~0u}};
__device__ __forceinline__ const uint4* win(const uint8_t* p, uint32_t at, uint32_t len) {
    return at < len ? (const uint4*)(p + at) : g_ff32;
}
__device__ __forceinline__ void ring_write16(uint32_t (*ring)[64], int lane, uint32_t pos, uint4 v) {
    const uint32_t j = (pos >> 2) & (RING_DW - 1);
    ring[j][lane] = v.x; ring[j + 1][lane] = v.y; ring[j + 2][lane] = v.z; ring[j + 3][lane] = v.w;
    if (j == 0) ring[RING_DW][lane] = v.x;   // mirror for wrap-around reads
}
__device__ __forceinline__ uint32_t ring_get4(uint32_t (*ring)[64], int lane, uint32_t bp) {
    const uint32_t j = (bp >> 2) & (RING_DW - 1);
    return __builtin_amdgcn_alignbyte(ring[j + 1][lane], ring[j][lane], bp & 3);
}
// the 32 staged bytes land in two register quads (no copies, so no wait after the issue)
template <class Q> __device__ __forceinline__ void stage_load(Q& q) {
    const uint4* w = win(q.p, q.sbase, q.len);
    q.Ta = w[0]; q.Tb = w[1];
}
// stripe-pass boundary: commit the staged 32 bytes when the ring has room, request the next 32
template <class Q> __device__ __forceinline__ void ring_boundary(uint32_t (*ring)[64], int lane, Q& q) {
    if (q.sbase != q.fill) { q.sbase = q.fill; stage_load(q); }   // after a synchronous top-up
    if (q.fill + 32 - q.bp <= 4 * RING_DW) {
        ring_write16(ring, lane, q.fill, q.Ta);
        ring_write16(ring, lane, q.fill + 16, q.Tb);
        q.fill += 32;
        q.sbase = q.fill;
        stage_load(q);
    }
}
// inside a step loop: synchronous top-up for a lane about to run dry
template <class Q> __device__ __forceinline__ void ring_topup(uint32_t (*ring)[64], int lane, Q& q, uint32_t low) {
    if (q.fill - q.bp < low) {
        ring_write16(ring, lane, q.fill, *win(q.p, q.fill, q.len));
        q.fill += 16;
    }
}


// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint64_t dil3(uint64_t u, uint64_t m, uint64_t d) {
    uint64_t t = u | m | d;
    return t | (t << 1) | (t >> 1);
}
// bits of the four stripe rows at column x (bit r = row r)
__device__ __forceinline__ uint32_t col4(uint64_t a, uint64_t b, uint64_t c, uint64_t d, uint32_t x) {
    return (uint32_t)((a >> x) & 1) | ((uint32_t)((b >> x) & 1) << 1) | ((uint32_t)((c >> x) & 1) << 2) |
           ((uint32_t)((d >> x) & 1) << 3);
}
enum { PH_FIND = 1, PH_SIGN = 2, PH_UNI1 = 4, PH_UNI2 = 8 };   // one-hot: the step tests bits

struct Rows22 {   // one stripe's rows: S1..S5 / N1..N5 (rows y0..y0+4), P/M/B (rows y0..y0+3)
    uint64_t s1, s2, s3, s4, s5, n1, n2, n3, n4, n5, p0, p1, p2, p3, m0, m1, m2, m3, b0, b1, b2, b3;
};
// rows of stripe y0 / plane `k` from the lane's scratch slab (consecutive words per field)
__device__ __forceinline__ void ld2(const uint64_t* p, uint64_t& a, uint64_t& b) {   // 16-byte aligned pair
    const ulonglong2 v = *(const ulonglong2*)p;
    a = v.x; b = v.y;
}
__device__ __forceinline__ void st2(uint64_t* p, uint64_t a, uint64_t b) { *(ulonglong2*)p = make_ulonglong2(a, b); }
// Only the rows the stripe-pass of type t (0 SP, 1 MR, 2 CL) reads are fetched: SP starts a
// plane (no plane-bit or visited rows) and ignores refinement rows; MR ignores signs; CL
// ignores refinement rows; the first cleanup pass (k == 0) has no plane or visited rows yet.
__device__ __forceinline__ void load_rows(Rows22& R, const uint64_t* WS, uint32_t k, uint32_t t, uint32_t y0) {
    const uint64_t* st = WS + 4 * y0;   // this stripe's line (y0 = 4 s)
    const uint64_t* bt = WS + WS_BITS + (size_t)k * 64 + y0;
    ld2(st + WS_S, R.s1, R.s2); ld2(st + WS_S + 2, R.s3, R.s4); R.s5 = st[16 + WS_S];
    if (t != 1) { ld2(st + WS_N, R.n1, R.n2); ld2(st + WS_N + 2, R.n3, R.n4); R.n5 = st[16 + WS_N]; }
    if (t != 0 && k != 0) { ld2(st + WS_P, R.p0, R.p1); ld2(st + WS_P + 2, R.p2, R.p3); ld2(bt, R.b0, R.b1); ld2(bt + 2, R.b2, R.b3); }
    if (t == 1) { ld2(st + WS_M, R.m0, R.m1); ld2(st + WS_M + 2, R.m2, R.m3); }
}

// next (plane, pass type, stripe) after (k, t, s); pass types 0 SP, 1 MR, 2 CL
__device__ __forceinline__ void next_pos3(uint32_t& k, uint32_t& t, uint32_t& s, uint32_t& pidx, uint32_t ns) {
    if (++s == ns) {
        s = 0; ++pidx;
        if (t == 2) { ++k; t = 0; } else ++t;
    }
}

struct Mq2 {
    uint64_t c;                  // bits 63:48 = Chigh; `avail` valid code bits below bit 48
    uint32_t a, avail;
    uint32_t bp, len, fill;      // byte position (last byte taken in), block length, ring fill position
    uint32_t nb4;                // bytes [bp, bp + 4)
    uint32_t sbase;              // staged bytes cover [sbase, sbase + 32)
    uint4 Ta, Tb;
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

// Two bytes at once when neither the last byte taken nor the next is 0xFF (both then carry 8
// bits, no marker can follow) and 16 bits fit; otherwise mq2_refill's one byte.  The refill
// loops take half the iterations.
__device__ __forceinline__ void mq2_refill2(Mq2& q, bool en) {
    const uint32_t cur = q.nb4 & 0xff, nxt = (q.nb4 >> 8) & 0xff, nn = (q.nb4 >> 16) & 0xff;
    const bool ff = cur == 0xff, stuck = ff & (nxt > 0x8f);
    const bool seven = ff & !stuck;
    const bool two = en & !ff & (nxt != 0xff) & (q.avail <= 32);
    const uint32_t v = two ? ((nxt << 8) | nn) : (en ? (stuck ? 0xffu : nxt) : 0u);
    const uint32_t sh = ((two ? 32u : 40u + (seven ? 1u : 0u)) - q.avail) & 63;
    q.c += (uint64_t)v << sh;
    q.avail += two ? 16u : (en ? (seven ? 7u : 8u) : 0u);
    const uint32_t adv = two ? 2u : ((en && !stuck) ? 1u : 0u);
    q.bp += adv;
    q.nb4 >>= 8 * adv;
}

struct Dec2Lds {
    uint32_t tab[96];                // (state, MPS) pair entries (mq_pair_entry)
    uint32_t ctx[19][64];            // per-lane context states as their (state, MPS) pair entries
    uint8_t zc[4][512];
    uint8_t sc[256];                 // index bit0 N-neg 1 N-sig 2 W-neg 3 W-sig 4 E-neg 5 E-sig 6 S-neg 7 S-sig
    uint32_t ring[RING_DW + 1][64];
    uint32_t sg[7 * 3][64];          // significance rows y0-1 .. y0+4 (+ a zero row), guarded: bit c+1 of the 96-bit row = column c
    uint32_t ng[7 * 3][64];          // sign rows (bits only where significant), same layout
    uint32_t mu[4 * 2][64];          // refined-in-an-earlier-plane rows y0 .. y0+3, plain 32-bit halves
    uint32_t bt[4 * 2][64];          // plane-bit rows y0 .. y0+3
    uint32_t pv[4 * 2][64];          // visited in SP of this plane, rows y0 .. y0+3 (SP stripe-passes)
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

// ------------------------------------------------------------------ solo decoding
// The wave's time is its heaviest lane's: the LL and low-resolution blocks (C2: 31.9 k decisions
// against a plateau of ~28 k for the level-1 bands; C3 without truncation 65 k against ~37 k) set
// the kernel time while a quarter of the SIMDs idle.  Those blocks are decoded by "solo" waves
// that run on the spare SIMDs, one block at a time: the control flow and the MQ registers are
// wave-uniform (scalar branches, SALU), so a decision costs what its own path needs instead of
// the lane-parallel step's every-case select chain.  The block's state sits in the lanes
// (lane = column x, bit y = row y): significance, sign, refined, visited-in-SP and the plane's
// bits, as 64-bit columns.  A stripe-pass packs each column's window into one dword per lane and
// walks the columns that have something to code (a ballot per stripe-pass) with three words in
// SGPRs (left, current, right); a column's word goes
// back with v_writelane and the stripe's rows are merged into the columns by VALU at its end.
// Context states, the (state, MPS) pair table and the ZC / SC rule tables live in VGPR lanes
// and are read with v_readlane.  Output: the plane-bit rows and the sign rows of the lane slab
// layout above (WS_BITS, WS_N), transposed with ballots, so k_t1_recon is shared.
// Same algorithm as the lane-parallel step (T1::decompress_cblk, T1.cpp:934-1446; Annex C.3 /
// D restated in oracle/j2k_oracle.cpp t1_decode_block), default code-block style only.
//
// Column word (per lane, rows relative to the stripe's first row y0):
//   bits 0-5   significance of rows y0-1 .. y0+4
//   bits 6-17  (significance, sign) pairs of rows y0-1 .. y0+4 (pair j at 6 + 2 j)
//   bits 18-21 visited in SP of this plane, rows y0 .. y0+3
//   bits 22-25 refined in an earlier plane
//   bits 26-29 bits of this plane
#define SW_PI 18
#define SW_MU 22
#define SW_BT 26
__device__ __forceinline__ uint32_t srl(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}
__device__ __forceinline__ uint32_t swl(uint32_t old, uint32_t val, uint32_t lane) {   // v_writelane_b32
    // (gfx9 reads one SGPR per VALU op besides M0: the lane select goes through M0)
    asm("v_writelane_b32 %0, %1, m0" : "+v"(old) : "s"(val), "{m0}"(lane));
    return old;
}
// rows y0-1 .. y0+4 of a column (bit 0 = row y0-1)
__device__ __forceinline__ uint32_t win6(uint64_t v, uint32_t y0) {
    return y0 ? (uint32_t)(v >> (y0 - 1)) & 0x3fu : (uint32_t)(v << 1) & 0x3fu;
}
__device__ __forceinline__ uint32_t spread6(uint32_t v) {   // bit j -> bit 2 j
    return (v & 1u) | ((v & 2u) << 1) | ((v & 4u) << 2) | ((v & 8u) << 3) | ((v & 16u) << 4) | ((v & 32u) << 5);
}
__device__ __forceinline__ uint32_t solo_prev(uint32_t v) {   // lane - 1's value, 0 at lane 0 (wave_shr:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t solo_next(uint32_t v) {   // lane + 1's value, 0 at lane 63 (wave_shl:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}
// ballot transpose: row y (bit x = lane x's bit y) into lane y of the result
__device__ __forceinline__ uint64_t rows_of(uint64_t col, uint32_t h, int lane) {
    uint32_t lo = 0, hi = 0;
    for (uint32_t y = 0; y < h; ++y) {
        const uint64_t r = __ballot((col >> y) & 1);
        lo = swl(lo, (uint32_t)r, y);
        hi = swl(hi, (uint32_t)(r >> 32), y);
    }
    return ((uint64_t)hi << 32) | lo;
}

// returns the decisions decoded (counted when STATS)
template <bool STATS>
__device__ uint32_t solo_block(const uint8_t* __restrict__ bytes, const GkBlock& B, uint64_t* __restrict__ WS, int lane) {
    const uint32_t numbps = B.numbps, npasses = B.numbps ? B.npasses : 0;
    if (!npasses) return 0;
    const uint32_t w = B.w, h = B.h, ns = (h + 3) >> 2, orient = B.orient & 3;
    // rule tables in lanes: ZC 8 entries of 4 bits per lane, index = left | centre << 3 | right << 6
    // (3 rows each, bit 0 = the row above); SC 4 entries of 8 bits per lane, index = (sig, sign)
    // pairs of N | W << 2 | S << 4 | E << 6
    uint32_t ZCL = 0, SCL = 0;
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t i = (uint32_t)lane * 8 + k;
        const uint32_t l = i & 7, c = (i >> 3) & 7, r = (i >> 6) & 7;
        // zc_rule: bit0 NW 1 N 2 NE 3 W 4 self 5 E 6 SW 7 S 8 SE
        const uint32_t f = (l & 1) | ((c & 1) << 1) | ((r & 1) << 2) | (((l >> 1) & 1) << 3) | (((c >> 1) & 1) << 4) |
                           (((r >> 1) & 1) << 5) | (((l >> 2) & 1) << 6) | (((c >> 2) & 1) << 7) | (((r >> 2) & 1) << 8);
        ZCL |= (uint32_t)zc_rule(orient, f) << (4 * k);
    }
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t i = (uint32_t)lane * 4 + k;
        // sc_rule: bit0 W-neg 1 W-sig 2 E-neg 3 E-sig 4 N-neg 5 N-sig 6 S-neg 7 S-sig
        const uint32_t N = i & 3, Wp = (i >> 2) & 3, S = (i >> 4) & 3, E = (i >> 6) & 3;
        const uint32_t f = (Wp >> 1) | ((Wp & 1) << 1) | ((E >> 1) << 2) | ((E & 1) << 3) | ((N >> 1) << 4) |
                           ((N & 1) << 5) | ((S >> 1) << 6) | ((S & 1) << 7);
        SCL |= (uint32_t)sc_rule(f) << (8 * k);
    }
    const uint32_t TAB0 = mq_pair_entry((uint32_t)lane), TAB1 = lane < MQ_PAIRS - 64 ? mq_pair_entry(64u + lane) : 0u;
    // mqc_resetstates (mqc_dec.cpp:121-130)
    uint32_t CTX = mq_pair_entry(2u * (lane == CTX_ZC ? 4u : (lane == CTX_AGG ? 3u : (lane == CTX_UNI ? 46u : 0u))));

    // compressed bytes: a 256-byte window in the lanes (4 per lane); bytes at or past the length
    // read 0xFF (the host pads every block with >= 32 bytes of 0xFF)
    const uint8_t* p = bytes + B.data_off;
    const uint32_t len = B.len;
    uint32_t wb = 0, BW = 0;
    auto load_window = [&](uint32_t at) {
        wb = at;
        const uint32_t o = at + 4u * (uint32_t)lane;
        BW = o < len ? *reinterpret_cast<const uint32_t*>(p + o) : 0xffffffffu;
    };
    load_window(0);
    // MQ code register (INITDEC / BYTEIN, Annex C.3.4-C.3.5, as Mq2 above): bits 63:48 = Chigh,
    // `avail` valid bits below; the queue starts with a 0 bit, then the bytes (7 bits after an
    // 0xFF, 1s for ever from a marker on)
    uint64_t c = 0;
    int32_t avail = -15;
    uint32_t a = 0x8000, bp = 0;
    bool prevff = false, ones = false;
    auto refill = [&]() {
        uint32_t off = bp - wb;
        if (off > 248) { load_window(bp); off = 0; }
        const uint32_t j = off >> 2, sh = (off & 3) * 8;
        const uint64_t two = ((uint64_t)srl(BW, j + 1) << 32) | srl(BW, j);
        const uint32_t word = (uint32_t)(two >> sh);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t b = (word >> (8 * k)) & 0xffu;
            if (!ones && prevff && b > 0x8f) ones = true;
            if (ones) {
                c += (uint64_t)0xffu << (40 - avail);
                avail += 8;
            } else if (prevff) {
                c += (uint64_t)b << (41 - avail);
                avail += 7;
                prevff = false;
                ++bp;
            } else {
                c += (uint64_t)b << (40 - avail);
                avail += 8;
                prevff = b == 0xffu;
                ++bp;
            }
        }
    };
    while (avail < 16) refill();
    uint32_t ndec = 0;
    auto tab = [&](uint32_t i) { return i < 64 ? srl(TAB0, i) : srl(TAB1, i - 64); };
    // DECODE (Annex C.3.2) with RENORMD as one shift
    auto dec = [&](uint32_t cx) -> uint32_t {
        if (STATS) ++ndec;
        const uint32_t e = srl(CTX, cx);
        const uint32_t qe = e & 0xffffu;
        uint32_t d = e >> 31;
        a -= qe;
        // lower sub-interval (Chigh < Qe): A = Qe, the exchange rule picks the symbol; upper: C -=
        // Qe, renormalisation only when A fell below 0x8000
        const uint32_t lower = (uint32_t)(c >> 48) < qe ? 1u : 0u;
        const uint32_t lps = lower ^ (a < qe ? 1u : 0u);
        const bool upd = lower || (a & 0x8000u) == 0;
        c -= lower ? 0ull : (uint64_t)qe << 48;
        a = lower ? qe : a;
        if (upd) {
            d ^= lps;
            CTX = swl(CTX, tab(lps ? (e >> 23) & 0x7fu : (e >> 16) & 0x7fu), cx);
            const uint32_t n = (uint32_t)__builtin_clz(a) - 16u;
            a <<= n;
            c <<= n;
            avail -= (int32_t)n;
            if (avail < 16) refill();
        }
        return d;
    };

    // block state: columns (bit y = row y)
    uint64_t SG = 0, NG = 0, PI = 0, MU = 0, BT = 0;
    uint32_t k = 0, t = 2;   // plane (0 = most significant) and pass type (0 SP, 1 MR, 2 CL)
    auto flush_plane = [&](uint32_t kk) {
        const uint64_t rows = rows_of(BT, h, lane);
        if ((uint32_t)lane < h) WS[WS_BITS + (size_t)kk * 64 + lane] = rows;
    };
    for (uint32_t pidx = 0; pidx < npasses && k < numbps; ++pidx) {
        for (uint32_t s = 0; s < ns; ++s) {
            const uint32_t y0 = 4 * s, nr = min(4u, h - y0);
            uint32_t W = win6(SG, y0) | (spread6(win6(SG, y0)) << 6) | (spread6(win6(NG, y0)) << 7) |
                         (((uint32_t)(PI >> y0) & 15u) << SW_PI) | (((uint32_t)(MU >> y0) & 15u) << SW_MU) |
                         (((uint32_t)(BT >> y0) & 15u) << SW_BT);
            // columns with something to code in this pass (SP: an insignificant sample with a
            // significant neighbour; MR: a significant sample not coded in SP; CL: an insignificant
            // sample not coded in SP); SP adds the column right of one that gains a significance
            uint64_t M;
            {
                const uint32_t S6 = W & 0x3fu, PI4 = (W >> SW_PI) & 15u, rows = (1u << nr) - 1u;
                const uint32_t D = solo_prev(S6) | solo_next(S6);
                const uint32_t nbr = D | (D >> 1) | (D >> 2) | S6 | (S6 >> 2);
                const uint32_t ins = ~(S6 >> 1) & rows;
                const uint32_t cr = t == 0 ? (nbr & ins) : (t == 1 ? ((S6 >> 1) & ~PI4 & rows) : (ins & ~PI4));
                M = __ballot(cr != 0 && (uint32_t)lane < w);
            }
            uint32_t Wl = 0, Wc = 0, Wr = 0, xp = 0xfffffffeu;   // no column before the first
            while (M) {
                const uint32_t x = (uint32_t)__builtin_ctzll(M);
                M &= M - 1;
                if (x == xp + 1) {
                    Wl = Wc; Wc = Wr;
                } else {
                    Wl = x ? srl(W, x - 1) : 0u;
                    Wc = srl(W, x);
                }
                Wr = x + 1 < w ? srl(W, x + 1) : 0u;
                const uint32_t sig0 = Wc & 0x1eu;
                auto zidx = [&](uint32_t i) {
                    return ((Wl >> i) & 7u) | (((Wc >> i) & 7u) << 3) | (((Wr >> i) & 7u) << 6);
                };
                // a decision 1 in ZC / run-length: the sign, then the sample is significant
                auto sign = [&](uint32_t i) {
                    const uint32_t si = ((Wc >> (6 + 2 * i)) & 0x33u) | (((Wl >> (8 + 2 * i)) & 3u) << 2) |
                                        (((Wr >> (8 + 2 * i)) & 3u) << 6);
                    const uint32_t sce = (srl(SCL, si >> 2) >> (8 * (si & 3))) & 0xffu;
                    const uint32_t sg = dec(CTX_SC + (sce & 15u)) ^ (sce >> 4);
                    Wc |= (1u << (1 + i)) | (1u << (8 + 2 * i)) | (sg << (9 + 2 * i)) | (1u << (SW_BT + i));
                };
                if (t == 0) {   // significance propagation (T1.cpp dec_sigpass)
                    for (uint32_t i = 0; i < nr; ++i) {
                        if ((Wc >> (1 + i)) & 1u) continue;
                        const uint32_t zi = zidx(i);
                        if (!zi) continue;
                        if (dec(CTX_ZC + ((srl(ZCL, zi >> 3) >> (4 * (zi & 7))) & 15u))) sign(i);
                        Wc |= 1u << (SW_PI + i);
                    }
                } else if (t == 1) {   // magnitude refinement (dec_refpass)
                    for (uint32_t i = 0; i < nr; ++i) {
                        if (((Wc >> (1 + i)) & 1u) == 0 || ((Wc >> (SW_PI + i)) & 1u)) continue;
                        const uint32_t cx = ((Wc >> (SW_MU + i)) & 1u) ? CTX_MAG + 2
                                            : ((zidx(i) & ~0x10u) ? CTX_MAG + 1 : CTX_MAG);
                        if (dec(cx)) Wc |= 1u << (SW_BT + i);
                        Wc |= 1u << (SW_MU + i);
                    }
                } else {   // cleanup (dec_clnpass), run-length mode on whole insignificant columns
                    uint32_t i = 0;
                    bool partial = false, skip = false;
                    if (nr == 4 && (((Wl | Wc | Wr) & 0x3fu) | ((Wc >> SW_PI) & 15u)) == 0) {
                        if (!dec(CTX_AGG)) {
                            skip = true;
                        } else {
                            i = dec(CTX_UNI) << 1;
                            i |= dec(CTX_UNI);
                            partial = true;
                        }
                    }
                    if (!skip) {
                        for (; i < nr; ++i) {
                            if (!partial) {
                                if (((Wc >> (1 + i)) & 1u) || ((Wc >> (SW_PI + i)) & 1u)) continue;
                                const uint32_t zi = zidx(i);
                                if (!dec(CTX_ZC + ((srl(ZCL, zi >> 3) >> (4 * (zi & 7))) & 15u))) continue;
                            }
                            partial = false;
                            sign(i);
                        }
                    }
                    Wc &= ~(15u << SW_PI);
                }
                W = swl(W, Wc, x);
                if (t == 0 && (Wc & 0x1eu) != sig0 && x + 1 < w) M |= 2ull << x;
                xp = x;
            }
            // the stripe's rows back into the columns
            const uint64_t m = ~((uint64_t)15 << y0);
            const uint32_t nb = ((W >> 9) & 1u) | ((W >> 10) & 2u) | ((W >> 11) & 4u) | ((W >> 12) & 8u);
            SG = (SG & m) | ((uint64_t)((W >> 1) & 15u) << y0);
            NG = (NG & m) | ((uint64_t)nb << y0);
            // (a cleanup pass clears the visited flags of every column, skipped ones included)
            PI = (PI & m) | (t == 2 ? 0ull : (uint64_t)((W >> SW_PI) & 15u) << y0);
            MU = (MU & m) | ((uint64_t)((W >> SW_MU) & 15u) << y0);
            BT = (BT & m) | ((uint64_t)((W >> SW_BT) & 15u) << y0);
        }
        if (t == 2) {
            flush_plane(k);
            BT = 0;
            ++k;
            t = 0;
        } else {
            ++t;
        }
    }
    if (t != 0 && k < numbps) flush_plane(k);   // a plane left after SP or MR
    // sign rows (where significant) in the stripe lines
    const uint64_t nrow = rows_of(NG, h, lane);
    if ((uint32_t)lane < h) WS[16 * (lane >> 2) + WS_N + (lane & 3)] = nrow;
    return ndec;
}

// TIMING (diagnostic build, GK_T1_STATS=2): shader-clock cycles spent in stripe-boundary
// events vs decision steps, summed into stats[4] / stats[5].
// MODE 0: decode; 1: also count decisions per lane (GK_T1_STATS); 2: also time events (=2).
// A workgroup is W independent waves (one per SIMD, W <= 4) and the launch pads its LDS to the
// CU's 160 KiB, so every decoding wave has its SIMD to itself (single waves per workgroup were
// placed two to a SIMD on some CUs while other SIMDs idled).
template <int MODE, int W>
__global__ __launch_bounds__(64 * W) void k_t1_dec2(const uint8_t* __restrict__ bytes,
                                                const GkBlock* __restrict__ blocks,
                                                const uint32_t* __restrict__ order, uint64_t* __restrict__ scratch,
                                                const uint64_t* __restrict__ wave_off, uint32_t nblocks,
                                                unsigned long long* __restrict__ stats, uint32_t kpark,
                                                uint32_t nsolo) {
    constexpr bool TIMING = MODE == 2, STATS = MODE >= 1;
    __shared__ Dec2Lds Lw[W];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    Dec2Lds& Ls = Lw[wv];
    const uint32_t gw = blockIdx.x * W + wv;          // global wave: 64 slots
    const uint32_t nwaves = (nblocks + 63) / 64;
    if (gw < nsolo) {   // solo wave: its blocks one after another (nsolo is a whole number of workgroups)
        // the wave index as a scalar, so everything derived from it stays in SGPRs and branches
        // stay scalar
        const uint32_t sgw = (uint32_t)__builtin_amdgcn_readfirstlane((int)gw);
        const uint64_t lstride = (wave_off[sgw + 1] - wave_off[sgw]) / 64;
        const uint64_t t0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
        uint32_t nd = 0;
        for (uint32_t i = 0; i < 64; ++i) {
            const uint32_t bid = order[sgw * 64 + i];
            if (bid == 0xffffffffu) break;
            const GkBlock B = blocks[bid];
            nd += solo_block<STATS>(bytes, B, scratch + wave_off[sgw] + i * lstride, lane);
        }
        // solo counters: decisions (all waves, busiest wave), cycles (all waves, longest wave
        // with its decisions: cycles << 20 | decisions)
        if (STATS && lane == 0 && nd) {
            atomicAdd(&stats[13], (unsigned long long)nd);
            atomicMax(&stats[14], (unsigned long long)nd);
            if (TIMING) {
                const uint64_t cyc = __builtin_amdgcn_s_memtime() - t0;
                atomicAdd(&stats[16], (unsigned long long)cyc);
                atomicMax(&stats[15], (unsigned long long)((cyc << 20) | min(nd, 0xfffffu)));
            }
        }
        return;
    }
    for (int i = lane; i < MQ_PAIRS; i += 64) Ls.tab[i] = mq_pair_entry((uint32_t)i);
    for (int i = lane; i < 2048; i += 64) Ls.zc[i >> 9][i & 511] = zc_rule((uint32_t)(i >> 9), (uint32_t)(i & 511));
    for (int i = lane; i < 256; i += 64)
        Ls.sc[i] = sc_rule((uint32_t)(((i >> 2) & 0xf) | ((i & 3) << 4) | (i & 0xc0)));
    const uint32_t slot = gw * 64 + lane;
    const uint32_t bid = slot < nblocks ? order[slot] : 0xffffffffu;   // empty slots: 0xffffffff
    const bool has = bid != 0xffffffffu;
    GkBlock B = {};
    if (has) B = blocks[bid];
    // this lane's scratch slab: the wave's region split into 64 equal slabs (host sizes
    // it for the wave's largest numbps and zero-fills it)
    const uint64_t lstride = gw < nwaves ? (wave_off[gw + 1] - wave_off[gw]) / 64 : 0;
    uint64_t* WS = scratch + (gw < nwaves ? wave_off[gw] : 0) + (size_t)lane * lstride;
    const uint32_t numbps = has ? B.numbps : 0, npasses = (has && B.numbps) ? B.npasses : 0;
    const uint32_t h = B.h, w = B.w;
    const uint64_t colmask = w >= 64 ? ~0ull : ((1ull << w) - 1);
    const uint32_t ns = (h + 3) >> 2;
    const uint8_t* zc = Ls.zc[B.orient & 3];
    for (int i = 0; i < 21; ++i) { Ls.sg[i][lane] = 0; Ls.ng[i][lane] = 0; }
    for (int i = 0; i < 8; ++i) { Ls.mu[i][lane] = 0; Ls.bt[i][lane] = 0; Ls.pv[i][lane] = 0; }
    // mqc_resetstates (mqc_dec.cpp:121-130): every context at state 0 except ZC0 = 4, AGG = 3, UNI = 46
    for (int c = 0; c < 19; ++c)
        Ls.ctx[c][lane] = mq_pair_entry(2 * (c == CTX_ZC ? 4 : (c == CTX_AGG ? 3 : (c == CTX_UNI ? 46 : 0))));
    uint32_t nstep = 0, nsym = 0, nevents = 0;
    unsigned long long cyc_ev = 0, cyc_step = 0, cyc_p[6] = {0, 0, 0, 0, 0, 0};
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
    // Candidates: C0..C3 are the stripe-pass's candidate rows at its start (static); the lane
    // walks them column by column: x = current column, nib = its rows still to code (the current
    // position included while in FIND), nn = rows of column x + 1 that SP propagation made
    // candidates.
    uint32_t nr = min(4u, h), x = 0xffffffffu, r = 0, ph = PH_FIND, rlhi = 0, nib = 0, nn = 0;
    uint32_t vr = (1u << nr) - 1;                 // valid rows of the stripe
    uint64_t C0, C1, C2, C3, CU, E;               // candidate rows, their union, run-length columns
    // lane masks: this stripe-pass set a bit in the plane's rows (write-back needed); the current
    // column gained a significance in this pass (a run-length test of the next column)
    uint32_t dirty = 0, colsig = 0;
    {
        const uint64_t v0 = nr > 0 ? colmask : 0, v1 = nr > 1 ? colmask : 0, v2 = nr > 2 ? colmask : 0,
                       v3 = nr > 3 ? colmask : 0;
        C0 = v0; C1 = v1; C2 = v2; C3 = v3;      // first CL: nothing significant yet
        CU = v0;
        E = (nr == 4) ? colmask : 0ull;
    }
    // The current decision's context cx and its state entry e are ready when a step starts; so
    // are, for the current position, the run-length flag, the 3x3 significance window fs and
    // the sign-context entry sce (for the SIGN decision that may follow).
    uint32_t cx = 0, e = 0, fs = 0, sce = 0;
    bool agg = false;
    // the entries of the two possible next contexts, read by the last step; the next step's R2
    // takes the one its decision selected (pend_b) when that step decided (pend_v)
    uint32_t eAp = 0, eBp = 0;
    uint32_t pend_v = 0, pend_b = 0, aggm = 0;   // lane masks
    // First position of column x + 1 or later (the next column with a stripe-start candidate, or
    // x + 1 when propagation gave it rows nn0), given the current column's rows nib0 still to code.
    auto next_position = [&](uint32_t nib0, uint32_t nn0, uint32_t& xA, uint32_t& nibA, uint32_t& nnA) {
        const uint32_t x1 = x + 1;
        const uint64_t rest = (CU >> (x1 & 63)) & (0ull - (uint64_t)(x1 < 64));
        const uint32_t xs = rest ? x1 + (uint32_t)__ffsll((long long)rest) - 1 : 64u;
        const uint32_t xadv = nn0 ? x1 : xs;
        const uint32_t nibadv = (col4(C0, C1, C2, C3, xadv & 63) & (0u - (uint32_t)(xadv < 64))) | nn0;
        const bool stay = nib0 != 0;
        xA = stay ? x : xadv;
        nibA = stay ? nib0 : nibadv;
        nnA = stay ? nn0 : 0u;
    };
    // The first position of a stripe-pass (lanes that `sel`): its window, contexts and entry.
    auto prep_stripe = [&](bool sel) {
        x = sel ? 0xffffffffu : x;
        uint32_t xA, nibA, nnA;
        next_position(0u, 0u, xA, nibA, nnA);
        const uint32_t rA = ((uint32_t)__ffs(nibA) - 1) & 3;
        const uint32_t Xc = xA & 63, dx = Xc >> 5, sx = Xc & 31, o0 = rA * 3 + dx;
        const uint32_t s0 = __builtin_amdgcn_alignbit(Ls.sg[o0 + 1][lane], Ls.sg[o0][lane], sx) & 7;
        const uint32_t s1 = __builtin_amdgcn_alignbit(Ls.sg[o0 + 4][lane], Ls.sg[o0 + 3][lane], sx) & 7;
        const uint32_t s2 = __builtin_amdgcn_alignbit(Ls.sg[o0 + 7][lane], Ls.sg[o0 + 6][lane], sx) & 7;
        const uint32_t n0 = __builtin_amdgcn_alignbit(Ls.ng[o0 + 1][lane], Ls.ng[o0][lane], sx) & 7;
        const uint32_t n1 = __builtin_amdgcn_alignbit(Ls.ng[o0 + 4][lane], Ls.ng[o0 + 3][lane], sx) & 7;
        const uint32_t n2 = __builtin_amdgcn_alignbit(Ls.ng[o0 + 7][lane], Ls.ng[o0 + 6][lane], sx) & 7;
        const uint32_t mub = (Ls.mu[rA * 2 + dx][lane] >> sx) & 1;
        const uint32_t fsA = s0 | (s1 << 3) | (s2 << 6), fnA = n0 | (n1 << 3) | (n2 << 6);
        const uint32_t scA = Ls.sc[(fsA & 0xaa) | ((fnA >> 1) & 0x55)];
        const bool aggA = (t == 2) & (((E >> Xc) & 1) != 0) & (nibA == 0xf);
        const uint32_t cxF = t == 1 ? (mub ? CTX_MAG + 2 : ((fsA & 0x1ef) ? CTX_MAG + 1 : CTX_MAG))
                                    : (aggA ? CTX_AGG : CTX_ZC + zc[fsA]);
        const uint32_t eF = Ls.ctx[cxF][lane];
        if (sel) {
            x = xA; r = rA; nib = nibA; nn = nnA; ph = PH_FIND; agg = aggA; fs = fsA; sce = scA; cx = cxF; e = eF;
            aggm = aggA ? ~0u : 0u;
            pend_v = 0;
            parked = parked || nibA == 0;   // a stripe-pass without candidates ends at once
        }
    };
    Rows22 X = {};
    {
        uint32_t k2 = k, t2 = t, s2 = s, p2 = pidx;
        next_pos3(k2, t2, s2, p2, ns);
        if (!done && p2 < npasses && k2 < numbps) load_rows(X, WS, k2, t2, 4 * s2);
    }

    // the lane with the most stripe-passes left (the wave lasts as long as it does), wave-uniform
    auto critical_lane = [&]() -> uint32_t {
        // work left: stripe-passes (default), compressed bytes (GK_T1DEC_CRIT=2) or 8 x bytes +
        // 4 x stripe-passes (GK_T1DEC_CRIT=3); kpark bits 10-11.  C2 max steps per wave:
        // 32,136 / 34,128 / 33,900 (round 4, with solo waves)
        const uint32_t sp = (npasses - pidx) * ns - s, nb = q.len > q.bp ? q.len - q.bp : 0u;
        const uint32_t mode = (kpark >> 10) & 3;
        const uint32_t rem = done ? 0u : min(mode == 0 ? sp : (mode == 1 ? nb : 8 * nb + 4 * sp), 0x3ffffffu);
        // wave max through DPP (row_shr 1/2/4/8, row_bcast 15/31): lane 63 ends with it
        uint32_t key = (rem << 6) | (uint32_t)lane;
        key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x111, 0xf, 0xf, false));
        key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x112, 0xf, 0xf, false));
        key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x114, 0xf, 0xf, false));
        key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x118, 0xf, 0xf, false));
        key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x142, 0xa, 0xf, false));
        key = max(key, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x143, 0xc, 0xf, false));
        return (uint32_t)__builtin_amdgcn_readlane((int)key, 63) & 63;
    };
    prep_stripe(!done);
    uint32_t crit_lane = critical_lane();

    while (__any(!done)) {
        // ---------------- stripe boundary for parked lanes (batched)
        const uint64_t parkedm = __ballot(parked);
        const uint32_t nparked = __popcll(parkedm);
        const uint32_t nactive = __popcll(__ballot(!done && !parked));
        uint64_t tev = 0;
        // a boundary event runs once kpark lanes wait, or at once when the lane with the most work
        // left is waiting: the wave's time is that lane's (it used to wait ~9 % of its steps)
        if (nparked && (nparked >= (kpark & 0xff) || nactive == 0 || ((parkedm >> crit_lane) & (kpark >> 8) & 1))) {
            ++nevents;
            if (TIMING) tev = __builtin_amdgcn_s_memtime();
            // everything the previous event issued has long landed: one explicit wait here
            // (seen by the compiler's counter model) keeps it from placing conservative waits
            // behind this event's own loads and stores
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
            if (!done && q.sbase == q.fill && q.fill + 32 - q.bp <= 4 * RING_DW) {
                ring_write16(Ls.ring, lane, q.fill, q.Ta);
                ring_write16(Ls.ring, lane, q.fill + 16, q.Tb);
                q.fill += 32;
            }
            // Write-back order.  The wave's vector memory counter covers loads and stores alike,
            // so a wait for a load issued after stores also waits for those stores.  Lanes of
            // blocks with >= 4 stripes therefore issue this event's loads (staged bytes, next
            // stripe prefetch) first and the write-back stores last; their prefetch never reads
            // rows written back in the same event.  Blocks with <= 3 stripes (prefetch rows that
            // overlap the finished stripe) store first, as program order then orders the reads.
            bool switched = false, late = false, wdirty = false;
            uint64_t W0 = 0, W1 = 0, W2 = 0, W3 = 0, W4 = 0, W5 = 0, W6 = 0, W7 = 0;   // finished stripe S1..S4, N1..N4
            uint64_t WB0 = 0, WB1 = 0, WB2 = 0, WB3 = 0, WP0 = 0, WP1 = 0, WP2 = 0, WP3 = 0;
            uint64_t WM0 = 0, WM1 = 0, WM2 = 0, WM3 = 0;
            uint32_t wy0 = 0, wk = 0, wt = 0, wmy = 0;
            bool wmu = false;
            uint64_t tp0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
            if (TIMING) cyc_p[3] += tp0 - tev;
            if (parked) {
                parked = false;
                switched = true;
                const uint32_t y0 = 4 * s;
                // the finished stripe: rows back to scratch
                const uint64_t S1 = g_get(Ls.sg, 1, lane), S2 = g_get(Ls.sg, 2, lane), S3 = g_get(Ls.sg, 3, lane),
                               S4 = g_get(Ls.sg, 4, lane);
                const uint64_t N1 = g_get(Ls.ng, 1, lane), N2 = g_get(Ls.ng, 2, lane), N3 = g_get(Ls.ng, 3, lane),
                               N4 = g_get(Ls.ng, 4, lane);
                const uint64_t B0 = h_get(Ls.bt, 0, lane), B1 = h_get(Ls.bt, 1, lane), B2 = h_get(Ls.bt, 2, lane),
                               B3 = h_get(Ls.bt, 3, lane);
                late = ns > 3;
                // rows a stripe-pass left unchanged are not stored: `dirty` marks a stripe-pass that
                // set a 1 bit in this plane's bit rows (a new significance in SP / CL, a refinement
                // 1 in MR); scratch starts zero-filled and SP is the first pass to touch a plane's
                // bit rows
                wdirty = dirty != 0;
                W0 = S1; W1 = S2; W2 = S3; W3 = S4; W4 = N1; W5 = N2; W6 = N3; W7 = N4;
                WB0 = B0; WB1 = B1; WB2 = B2; WB3 = B3;
                const uint64_t P0 = h_get(Ls.pv, 0, lane), P1 = h_get(Ls.pv, 1, lane), P2 = h_get(Ls.pv, 2, lane),
                               P3 = h_get(Ls.pv, 3, lane);
                WP0 = P0; WP1 = P1; WP2 = P2; WP3 = P3;
                wy0 = y0; wk = k; wt = t;
                if (!late) {
                    uint64_t* sgp = WS + 4 * y0 + WS_S;
                    uint64_t* ngp = WS + 4 * y0 + WS_N;
                    uint64_t* pip = WS + 4 * y0 + WS_P;
                    uint64_t* btp = WS + WS_BITS + (size_t)k * 64 + y0;
                    if (t != 1 && wdirty) {   // MR changes neither significance nor signs
                        st2(sgp, S1, S2); st2(sgp + 2, S3, S4);
                        st2(ngp, N1, N2); st2(ngp + 2, N3, N4);
                    }
                    if (t == 0) { st2(pip, P0, P1); st2(pip + 2, P2, P3); }
                    if (wdirty) { st2(btp, B0, B1); st2(btp + 2, B2, B3); }
                }
                if (TIMING) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc_p[0] += t - tp0; tp0 = t; }
                next_pos3(k, t, s, pidx, ns);
                done = pidx >= npasses || k >= numbps;
                // New stripe rows come from the prefetch X, issued when the finished stripe
                // started.  For 1-stripe blocks (and 2-stripe blocks at a pass change) that
                // prefetch overlapped the finished stripe's rows, so those lanes reload them
                // now, after the write-back above (rare: only the smallest bands).
                const bool resync = !done && (ns == 1 || (ns == 2 && s == 0));
                if (__any(resync)) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (resync) load_rows(X, WS, k, t, 4 * s);
                }
                const bool newplane = t == 0 || k == 0;
                const uint64_t nS0 = s ? S4 : 0ull, nN0 = s ? N4 : 0ull;
                const uint64_t nS1 = X.s1, nS2 = X.s2, nS3 = X.s3, nS4 = X.s4, nS5 = X.s5;
                const uint64_t nN1 = X.n1, nN2 = X.n2, nN3 = X.n3, nN4 = X.n4, nN5 = X.n5;
                const uint64_t nM0 = X.m0, nM1 = X.m1, nM2 = X.m2, nM3 = X.m3;
                const uint64_t nB0 = newplane ? 0ull : X.b0, nB1 = newplane ? 0ull : X.b1,
                               nB2 = newplane ? 0ull : X.b2, nB3 = newplane ? 0ull : X.b3;
                const uint64_t pP0 = t == 0 ? 0ull : X.p0, pP1 = t == 0 ? 0ull : X.p1, pP2 = t == 0 ? 0ull : X.p2,
                               pP3 = t == 0 ? 0ull : X.p3;
                g_put(Ls.sg, 0, lane, nS0); g_put(Ls.sg, 1, lane, nS1); g_put(Ls.sg, 2, lane, nS2);
                g_put(Ls.sg, 3, lane, nS3); g_put(Ls.sg, 4, lane, nS4); g_put(Ls.sg, 5, lane, nS5);
                g_put(Ls.ng, 0, lane, nN0); g_put(Ls.ng, 1, lane, nN1); g_put(Ls.ng, 2, lane, nN2);
                g_put(Ls.ng, 3, lane, nN3); g_put(Ls.ng, 4, lane, nN4); g_put(Ls.ng, 5, lane, nN5);
                h_put(Ls.mu, 0, lane, nM0); h_put(Ls.mu, 1, lane, nM1); h_put(Ls.mu, 2, lane, nM2); h_put(Ls.mu, 3, lane, nM3);
                h_put(Ls.bt, 0, lane, nB0); h_put(Ls.bt, 1, lane, nB1); h_put(Ls.bt, 2, lane, nB2); h_put(Ls.bt, 3, lane, nB3);
                h_put(Ls.pv, 0, lane, 0); h_put(Ls.pv, 1, lane, 0); h_put(Ls.pv, 2, lane, 0); h_put(Ls.pv, 3, lane, 0);
                if (TIMING) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc_p[1] += t - tp0; tp0 = t; }
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
                CU = C0 | C1 | C2 | C3;
                E = (t == 2 && nr == 4) ? (C0 & C1 & C2 & C3 & ~dil3(nS0 | nS1, nS2 | nS3, nS4 | nS5)) : 0ull;
                // SP: visited = the positions it codes (pv rows in LDS); MR: refined = old | coded now
                // MR refines every candidate: the rows after this pass, stored with the write-back
                wmu = t == 1; wmy = ny0;
                WM0 = nM0 | C0; WM1 = nM1 | C1; WM2 = nM2 | C2; WM3 = nM3 | C3;
                if (wmu && !late) {
                    uint64_t* mup = WS + 4 * ny0 + WS_M;
                    st2(mup, WM0, WM1); st2(mup + 2, WM2, WM3);
                }
                dirty = 0; colsig = 0; nn = 0; ph = PH_FIND;
                if (TIMING) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc_p[2] += t - tp0; tp0 = t; }
            }
            prep_stripe(switched && !done);
            crit_lane = critical_lane();
            // stage the next ring bytes (lanes whose fill point moved) and prefetch the next
            // stripe of the lanes that switched (the others keep theirs): no re-reads
            uint64_t tq0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
            if (q.sbase != q.fill) { q.sbase = q.fill; stage_load(q); }
            if (TIMING) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc_p[4] += t - tq0; tq0 = t; }
            uint32_t k2 = k, t2 = t, s2 = s, p2 = pidx;
            next_pos3(k2, t2, s2, p2, ns);
            if (switched && !done && p2 < npasses && k2 < numbps)
                load_rows(X, WS, k2, t2, 4 * s2);
            if (late) {
                uint64_t* sgp = WS + 4 * wy0 + WS_S;
                uint64_t* ngp = WS + 4 * wy0 + WS_N;
                uint64_t* pip = WS + 4 * wy0 + WS_P;
                uint64_t* btp = WS + WS_BITS + (size_t)wk * 64 + wy0;
                if (wt != 1 && wdirty) {
                    st2(sgp, W0, W1); st2(sgp + 2, W2, W3);
                    st2(ngp, W4, W5); st2(ngp + 2, W6, W7);
                }
                if (wt == 0) { st2(pip, WP0, WP1); st2(pip + 2, WP2, WP3); }
                if (wdirty) { st2(btp, WB0, WB1); st2(btp + 2, WB2, WB3); }
                if (wmu && !done) {
                    uint64_t* mup = WS + 4 * wmy + WS_M;
                    st2(mup, WM0, WM1); st2(mup + 2, WM2, WM3);
                }
            }
            if (TIMING) { const uint64_t t = __builtin_amdgcn_s_memtime(); cyc_p[5] += t - tq0; }
            if (TIMING) { const uint64_t t1 = __builtin_amdgcn_s_memtime(); cyc_ev += t1 - tev; tev = t1; }
        }
        if (TIMING && !tev) tev = __builtin_amdgcn_s_memtime();
        // ---------------- decisions: T1DEC_UNROLL steps per loop iteration.  The stripe-boundary
        // test at the loop head then runs once per group, and more lanes are parked when it does,
        // so events are fewer and larger (C2: 3325 -> 1891 per wave); parked lanes idle meanwhile
        // The code register is refilled to > 40 bits once per group (at most 6 bytes); a step
        // then takes ring bytes only in a renormalisation burst (at most 2: a decision needs 16
        // bits and leaves at least 1), and ring_get4 looks 4 ahead: 6 + 2 * T1DEC_UNROLL + 4
        // bytes must be staged per group (kMargin).  q.nb4 stays valid while bp does not move.
        constexpr uint32_t kMargin = (6 + 2 * T1DEC_UNROLL + 4 + 15) / 16 * 16;
        static_assert(kMargin + 16 + 32 <= 4 * RING_DW, "ring top-up margin");
        while (__any(q.fill - q.bp < kMargin)) ring_topup(Ls.ring, lane, q, kMargin);
        while (__any(!done && q.avail <= 40)) {
            mq2_refill2(q, !done && q.avail <= 40);
            q.nb4 = ring_get4(Ls.ring, lane, q.bp);
        }
        // lane masks constant over the group: active, pass type (t: 0 SP, 1 MR, 2 CL)
        uint32_t actm = (!done && !parked) ? ~0u : 0u;
        const uint32_t mSP = mlt(t, 1), mMR = mbit(t, 0), mCL = mbit(t, 1);
        uint32_t parkm = 0;
        // need: some lane must refill its code register before its next decision (computed at the
        // end of the previous step, so the branch does not wait)
        bool need = __any((actm != 0) & (q.avail < 16));
        auto step = [&]() __attribute__((always_inline)) {
            // ---------------- one decision per active lane.  While it is decoded, the next step's
            // context is fetched for both outcomes: A, the next FIND position (where a 0 leads, or
            // where MR and SIGN lead anyway) with its significance window, LUT entry and context
            // entry, and B (SIGN after a ZC 1, UNI1 after a run-length 1) with its entry.  The
            // decision then only selects, so the LDS round trips are off the chain from one
            // decision to the next.  The step is one basic block cut into regions by scheduling
            // fences, ordered so that a region's LDS reads land while the next region computes:
            //   R1 position A, window reads | R2 this decision | R3 windows -> LUT reads |
            //   R4 state updates, context write-back | R5 contexts of A and B, entry reads |
            //   R6 next state (the entry is selected in the next step's R2)
            // SIGN after UNI2 (a run-length interruption) is a B outcome with a fixed context: the
            // run-length column and its neighbours are insignificant (the aggregation condition),
            // and so are the rows the run covered, so the sample's sign context is that of an
            // all-insignificant neighbourhood (SC index 0: context CTX_SC, no sign flip).
            ++nstep;
            if (__builtin_expect(need, 0)) {
                while (__any((actm != 0) & (q.avail < 16))) {   // a burst of long renormalisations
                    mq2_refill2(q, (actm != 0) & (q.avail < 16));
                    q.nb4 = ring_get4(Ls.ring, lane, q.bp);
                }
            }
            // ---- R1
            const uint32_t mF = mbit(ph, 0), mS = mbit(ph, 1), mU1 = mbit(ph, 2), mU2 = mbit(ph, 3);
            // SIGN: the sample becomes significant now (its sign bit follows the decision)
            const uint32_t gx = x + 1, gd = (gx >> 5) & 3, gb = 1u << (gx & 31);
            const uint32_t sgn = actm & mS;
            atomicOr(&Ls.sg[(r + 1) * 3 + gd][lane], gb & sgn);
            const uint32_t spn = sgn & mSP;   // SP propagation from the new significance
            const uint32_t nf = ~fs;
            const uint32_t ca = (((nf >> 7) & 1) << (r + 1)) & vr & spn;
            const uint32_t t3 = ((nf >> 2) & 1) | ((nf >> 4) & 2) | ((nf >> 6) & 4);
            const uint32_t cb = ((t3 << r) >> 1) & vr & spn & mlt(gx, w);
            const uint32_t nib0 = bsel(mF, nib & ~(1u << r) & ~aggm, nib | ca);
            const uint32_t nn0 = nn | cb;
            const uint32_t cs0 = colsig | sgn;
            // next position: the current column's next row, else x + 1 (propagated rows) or the
            // next column with a stripe-start candidate
            const uint32_t x1 = x + 1;
            const uint64_t rest = CU >> (x1 & 63);
            const uint32_t in64 = mlt(x1, 64);
            const uint32_t frel = min(ffbl((uint32_t)rest & in64),   // first set bit, ~0 if none
                                      min(ffbl((uint32_t)(rest >> 32) & in64), 0xffffffdfu) + 32u);
            const uint32_t xs = min(x1 + min(frel, 64u), 64u);
            const uint32_t xadv = bsel(mnz(nn0), x1, xs);
            const uint32_t nibadv = (col4(C0, C1, C2, C3, xadv & 63) & mlt(xadv, 64)) | nn0;
            const uint32_t stay = mnz(nib0);
            const uint32_t xA = bsel(stay, x, xadv), nibA = bsel(stay, nib0, nibadv), nnA = nn0 & stay;
            const uint32_t rA = (uint32_t)ffbl(nibA) & 3;
            // significance window of A; sign window of the current position (its sign context)
            const uint32_t XA = xA & 63, dA = XA >> 5, sA = XA & 31, oA = rA * 3 + dA;
            const uint32_t g0a = Ls.sg[oA][lane], g0b = Ls.sg[oA + 1][lane], g1a = Ls.sg[oA + 3][lane],
                           g1b = Ls.sg[oA + 4][lane], g2a = Ls.sg[oA + 6][lane], g2b = Ls.sg[oA + 7][lane];
            const uint32_t muw = Ls.mu[rA * 2 + dA][lane];
            const uint32_t Xc = x & 63, dC = Xc >> 5, sC = Xc & 31, oC = r * 3 + dC;
            const uint32_t h0a = Ls.ng[oC][lane], h0b = Ls.ng[oC + 1][lane], h1a = Ls.ng[oC + 3][lane],
                           h1b = Ls.ng[oC + 4][lane], h2a = Ls.ng[oC + 6][lane], h2b = Ls.ng[oC + 7][lane];
            __builtin_amdgcn_sched_barrier(0);
            // ---- R2: the entry selected by the last decision; DECODE (Annex C.3.2; RENORMD as one shift)
            e = bsel(pend_v, bsel(pend_b, eBp, eAp), e);
            const uint32_t tM = Ls.tab[(e >> 16) & 0x7f], tL = Ls.tab[(e >> 23) & 0x7f];   // MPS / LPS successor pairs
            const uint32_t mps = e >> 31, qe = e & 0xffff;
            const uint32_t chi = (uint32_t)(q.c >> 32);
            const uint32_t a1 = q.a - qe;
            const uint32_t lower = mlt(chi >> 16, qe);
            const uint32_t fast = ~lower & mbit(a1, 15);
            const uint32_t mpsp = lower ^ ~mlt(a1, qe);      // exchange rule
            const uint32_t d = mps ^ (~(fast | mpsp) & 1);
            const uint32_t upd = actm & ~fast;
            const uint32_t an = bsel(actm, bsel(lower, qe, a1), q.a);
            const uint32_t ch = chi - ((qe << 16) & actm & ~lower);
            const uint32_t nsh = (ffbh(an) - 16) & upd;   // an != 0
            q.a = an << nsh;
            q.c = (((uint64_t)ch << 32) | (uint32_t)q.c) << nsh;
            q.avail -= nsh;
            if (STATS) nsym += actm & 1;
            __builtin_amdgcn_sched_barrier(0);
            // ---- R3: windows -> LUT reads (zero coding of A, sign context of the current position)
            const uint32_t fsA = (__builtin_amdgcn_alignbit(g0b, g0a, sA) & 7) | ((__builtin_amdgcn_alignbit(g1b, g1a, sA) & 7) << 3) |
                                 ((__builtin_amdgcn_alignbit(g2b, g2a, sA) & 7) << 6);
            const uint32_t fnC = (__builtin_amdgcn_alignbit(h0b, h0a, sC) & 7) | ((__builtin_amdgcn_alignbit(h1b, h1a, sC) & 7) << 3) |
                                 ((__builtin_amdgcn_alignbit(h2b, h2a, sC) & 7) << 6);
            const uint32_t zcA = zc[fsA];
            const uint32_t sce = Ls.sc[(fs & 0xaa) | ((fnC >> 1) & 0x55)];
            __builtin_amdgcn_sched_barrier(0);
            // ---- R4: state updates: plane bit (significance or refinement 1), visited in SP; the
            // context's new entry written back (the reads of R5 come after it)
            const uint32_t md = mbit(d, 0);
            const uint32_t pb = sgn | (actm & mF & mMR & md);
            const uint32_t dx0 = (x >> 5) & 1, bx = 1u << (x & 31);
            atomicOr(&Ls.bt[r * 2 + dx0][lane], bx & pb);
            atomicOr(&Ls.pv[r * 2 + dx0][lane], bx & actm & mF & mSP);
            dirty |= pb;
            // next state: FIND at A after a 0 (FIND), always after MR and SIGN; SIGN after a ZC 1;
            // UNI1 after a run-length 1; UNI2 after UNI1; SIGN at row 2 rlhi + d after UNI2
            const uint32_t takeB = mF & ~mMR & md;
            const uint32_t toA = (mF & ~takeB) | mS;
            const uint32_t rr = (rlhi << 1) | d;
            const uint32_t nph = bsel(toA, PH_FIND, bsel(mF, bsel(aggm, PH_UNI1, PH_SIGN), bsel(mU1, PH_UNI2, PH_SIGN)));
            const uint32_t consumed = bsel(mF & ~aggm, 1u << r, ((2u << rr) - 1) & mU2);
            const uint32_t ne = bsel(mpsp, tM, tL);
            Ls.ctx[cx][lane] = bsel(upd, ne, e);
            // some lane must refill its code register, or fetch a SIGN context after UNI2, before its
            // next decision: decided here so the next step's branch does not wait for the compare
            need = __any((actm & mlt(q.avail, 16)) != 0);
            __builtin_amdgcn_sched_barrier(0);
            // ---- R5: the sign, the contexts of A and B and their entries
            const uint32_t negs = sgn & mbit(d ^ (sce >> 4), 0);
            atomicOr(&Ls.ng[(r + 1) * 3 + gd][lane], gb & negs);
            // a column starts in run-length mode when it was eligible at stripe start, is untouched
            // and its left neighbour column gained no significance in this pass.  A run-length
            // column is a new column (nibA = all rows), and the columns between this one and it
            // had no candidates, so only this column (the neighbour iff XA = x + 1) can have gained one
            const uint32_t aggA = mCL & mbit((uint32_t)(E >> XA), 0) & mbit(nibA + 1, 4) & ~(cs0 & mz(XA ^ gx));
            const uint32_t cxM = bsel(mbit(muw, sA), CTX_MAG + 2, bsel(mnz(fsA & 0x1ef), CTX_MAG + 1, CTX_MAG));
            const uint32_t cxF = bsel(mMR, cxM, bsel(aggA, CTX_AGG, CTX_ZC + zcA));
            const uint32_t cxA = bsel(mU1, CTX_UNI, cxF);
            const uint32_t cxB = bsel(mU2, CTX_SC, bsel(aggm, CTX_UNI, CTX_SC + (sce & 15)));
            eAp = Ls.ctx[cxA][lane];
            eBp = Ls.ctx[cxB][lane];
            __builtin_amdgcn_sched_barrier(0);
            // ---- R6: next state (lanes that did not decide keep cx / e and are parked or done, so
            // their other fields are rebuilt at the next stripe boundary)
            fs = bsel(toA, fsA, fs);
            colsig = cs0 & ~(toA & mnz(xA ^ x));   // a new column has gained nothing yet
            aggm = bsel(toA, aggA, aggm);
            x = bsel(toA, xA, x);
            r = bsel(toA, rA, bsel(mU2, rr, r));
            nn = bsel(toA, nnA, nn);
            nib = bsel(toA, nibA, nib & ~consumed);
            rlhi = bsel(mU1, d, rlhi);
            ph = nph;
            const uint32_t np = actm & toA & ~mnz(nibA);   // no position left: the stripe-pass ends
            parkm |= np;
            cx = bsel(actm, bsel(takeB | mU2, cxB, cxA), cx);
            pend_v = actm; pend_b = takeB | mU2;
            actm &= ~np;
            __builtin_amdgcn_sched_barrier(0);
        };
#pragma unroll
        for (int us = 0; us < T1DEC_UNROLL / 2; ++us) step();
        // half-way through the group: when the lane with the most work left has parked, the group
        // ends here and its boundary event runs now (that lane used to wait for the group's end,
        // ~6 steps per stripe-pass, ~8 % of its wave's steps); kpark bit 9.  Tests at every
        // quarter were measured in round 4: 32,136 -> 32,049 steps but 20.5 -> 21.1 ms (the two
        // extra tests and the broken-up unrolled body cost more than the steps saved)
        if (!((kpark >> 9) & 1) || __builtin_amdgcn_readlane((int)parkm, (int)crit_lane) == 0) {
#pragma unroll
            for (int us = T1DEC_UNROLL / 2; us < T1DEC_UNROLL; ++us) step();
        }
        parked = parked || parkm != 0;
        agg = aggm != 0;
        if (TIMING) cyc_step += __builtin_amdgcn_s_memtime() - tev;
    }
    unsigned long long cp[6] = {0, 0, 0, 0, 0, 0};
    if (TIMING) {   // the parked block runs on the parked lanes only: take the max over lanes per event
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            cp[i] = cyc_p[i];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) cp[i] = max(cp[i], (unsigned long long)__shfl_xor(cp[i], o));
        }
    }
    if (stats) {
        unsigned long long tot = nsym;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        if (lane == 0) {
            if (TIMING) { atomicAdd(&stats[4], cyc_ev); atomicAdd(&stats[5], cyc_step); }
            if (TIMING)
                for (int i = 0; i < 6; ++i) atomicAdd(&stats[6 + i], cp[i]);
            atomicAdd(&stats[3], (unsigned long long)nevents);
            atomicAdd(&stats[0], (unsigned long long)nstep); atomicAdd(&stats[1], tot);
            atomicMax(&stats[2], (unsigned long long)nstep);
        }
        if (stats) {   // the busiest lane of the kernel: its decisions, and the steps of its wave
            unsigned long long mx = nsym;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned long long)__shfl_xor(mx, o));
            if (lane == 0) atomicMax(&stats[12], (mx << 32) | nstep);
        }
    }
}

// Reconstruction + dequantisation: wave per block, lane = column.
// Job q reconstructs block ids[q], whose decoder lane was pos[q]. The block's
// significant bit-plane rows and sign rows are staged once through LDS with
// coalesced row loads (lane = row); the column extraction then reads them as
// LDS broadcasts instead of one uniform global load per (row, plane).
// The staging holds the launch's largest plane count (dynamic LDS: 16 KB for 32 planes capped
// a CU at 9 such waves; C2's 11 planes take 6 KB).
__global__ __launch_bounds__(64) void k_t1_recon(const GkBlock* __restrict__ blocks, const uint32_t* __restrict__ ids,
                                                 const uint32_t* __restrict__ pos,
                                                 const uint64_t* __restrict__ scratch,
                                                 const uint64_t* __restrict__ wave_off, int32_t* __restrict__ coef,
                                                 uint32_t nblocks, uint32_t npmax) {
    extern __shared__ uint64_t Lrec[];
    uint64_t* Lr = Lrec;                 // npmax plane rows x 64
    uint64_t* Ls = Lrec + npmax * 64;    // sign rows
    const uint32_t q = blockIdx.x;
    if (q >= nblocks) return;
    const int x = threadIdx.x;
    const GkBlock B = blocks[ids[q]];
    const uint32_t slot = pos[q], ln = slot & 63;
    const uint64_t lstride = (wave_off[(slot >> 6) + 1] - wave_off[slot >> 6]) / 64;
    const uint64_t* WS = scratch + wave_off[slot >> 6] + (size_t)ln * lstride;
    const bool irrev = B.flags & 1;
    const uint32_t rs = B.flags >> 3;   // ROI shift of the component (RGN)
    float* fcoef = reinterpret_cast<float*>(coef);
    const uint32_t numbps = B.numbps, npasses = B.npasses, h = B.h;
    // last decoded pass k = npasses-1: pass k>0 belongs to plane numbps-1-(k+2)/3, type (k+2)%3
    int bpl = 0, t = 2;
    const bool any = npasses && numbps;
    if (any) {
        int k = (int)npasses - 1;
        if (k > 3 * (int)numbps - 3) k = 3 * (int)numbps - 3;
        bpl = (int)numbps - 1 - (k + 2) / 3;
        t = (k + 2) % 3;
        const int np = min((int)numbps - bpl, (int)npmax);   // planes numbps-1 .. bpl, row i = numbps-1-p
        if (x < (int)h) {
#pragma unroll 4
            for (int i = 0; i < np; ++i) Lr[i * 64 + x] = WS[WS_BITS + (size_t)i * 64 + x];
            Ls[x] = WS[4 * (x & ~3) + WS_N + (x & 3)];
        }
    }
    __syncthreads();
    if (x >= (int)B.w) return;
    const int np = min((int)numbps - bpl, (int)npmax);
    // the lane's half of each 64-bit row: one 32-bit LDS read and a bit-field extract per plane
    const uint32_t* Lh = reinterpret_cast<const uint32_t*>(Lr) + (x >> 5);
    const uint32_t xb = x & 31;
    for (uint32_t y = 0; y < h; ++y) {
        int32_t v = 0;
        if (any) {
            uint32_t M = 0;
            for (int i = 0; i < np; ++i) M |= __builtin_amdgcn_ubfe(Lh[2 * (i * 64 + y)], xb, 1) << ((int)numbps - 1 - i);
            if (M) {
                int qq = (t == 0 && (M >> (bpl + 1)) != 0) ? bpl + 1 : bpl;
                int32_t mag = (int32_t)(((M >> qq) << 1 | 1) << qq);
                bool ng = (Ls[y] >> x) & 1;
                v = ng ? -mag : mag;
            }
        }
        size_t o = B.band_off + (size_t)y * B.stride + x;
        if (rs) {   // RoiShiftFilter / RoiScaleFilter (PostDecompressFilters.h:7-72)
            const int32_t m = v < 0 ? -v : v;
            if (m >= (1 << rs)) v = v < 0 ? -(m >> rs) : (m >> rs);
        }
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
// max steps per wave, steps, symbols, solo decisions, solo decisions of the busiest solo wave (GK_T1_STATS)
static uint64_t g_last_stats[5] = {0, 0, 0, 0, 0};
void gk_t1dec_stats(uint64_t out[5]) { for (int i = 0; i < 5; ++i) out[i] = g_last_stats[i]; }
// Solo waves for a decode of nblocks blocks at `lanes` per wave: the SIMDs the lane-parallel
// waves leave (4 per CU), in whole workgroups of 12 waves (3 or 4 per group), at most 512.
// GK_T1DEC_SOLO=n forces n solo blocks, one per wave (0: none); GK_T1DEC_SOLO_R sets the cost
// ratio the host packs with (gk_engine.cpp: a lane-parallel wave's cycles per decision of its
// busiest lane over a solo wave's cycles per decision; C2 measured ~1,675 / 572).
GkSoloPlan gk_t1dec_solo_plan(uint32_t nblocks, uint32_t lanes) {
    static int ncu = -1, force = -2;
    static float ratio = 2.5f;
    if (ncu < 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            n = 0;
        ncu = n;
        const char* v = getenv("GK_T1DEC_SOLO");
        force = v ? atoi(v) : -1;
        if (const char* r = getenv("GK_T1DEC_SOLO_R")) ratio = (float)atof(r);
    }
    GkSoloPlan sp{0, -1, ratio};
    if (force >= 0) {
        sp.forced = (int)std::min<uint32_t>((uint32_t)force, nblocks);
        sp.waves = ((uint32_t)sp.forced + 11) / 12 * 12;
        return sp;
    }
    const uint32_t simds = 4u * (uint32_t)ncu, nw = (nblocks + lanes - 1) / lanes;
    if (nw + 12 > simds || nblocks < 8) return sp;
    sp.waves = std::min<uint32_t>((simds - nw) / 12 * 12, 512u);
    return sp;
}

void gk_launch_t1_dec(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, const uint32_t* order,
                      uint64_t* scratch, const uint64_t* wave_off, uint32_t nblocks, uint32_t nsolo) {
    if (!nblocks) return;
    static unsigned long long* stats = nullptr;
    const char* sv = getenv("GK_T1_STATS");
    const bool want = sv != nullptr, timing = sv && atoi(sv) == 2;
    if (want && !stats) { (void)hipMalloc(&stats, 256); }
    if (want) (void)hipMemsetAsync(stats, 0, 256, st);
    static int kpark = -1;
    if (kpark < 0) {
        const char* kp = getenv("GK_T1DEC_PARK");   // parked lanes that trigger a stripe boundary
        kpark = kp ? atoi(kp) : 16;
        // GK_T1DEC_CRIT=0: no event for the lane with the most work left alone (bit 8 of kpark)
        const char* kc = getenv("GK_T1DEC_CRIT");
        if (!kc || atoi(kc)) kpark |= 0x100;
        if (kc && atoi(kc) >= 2) kpark |= (atoi(kc) - 1) << 10;
        // GK_T1DEC_MID=0: no half-group exit when that lane has parked (bit 9)
        const char* km = getenv("GK_T1DEC_MID");
        if (!km || atoi(km)) kpark |= 0x200;
    }
    const uint32_t nwaves = (nblocks + 63) / 64;
    auto launch = [&](auto kern, uint32_t W, unsigned long long* stp) {
        const uint32_t ngroups = (nwaves + W - 1) / W;
        const size_t pad = W * sizeof(Dec2Lds) < 163840 ? 163840 - W * sizeof(Dec2Lds) : 0;
        hipLaunchKernelGGL(kern, dim3(ngroups), dim3(64 * W), pad, st, bytes, blocks, order, scratch, wave_off, nblocks,
                           stp, (uint32_t)kpark, nsolo);
    };
    // four waves per workgroup (three per group was measured: C2 decode 20.5 -> 31.9 ms, the
    // groups no longer fit one per CU next to the solo waves' groups)
    if (timing)
        launch(k_t1_dec2<2, 4>, 4, stats);
    else if (want)
        launch(k_t1_dec2<1, 4>, 4, stats);
    else
        launch(k_t1_dec2<0, 4>, 4, nullptr);
    if (want) {
        unsigned long long h[32];
        (void)hipMemcpyAsync(h, stats, 256, hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
        g_last_stats[0] = h[2]; g_last_stats[1] = h[0]; g_last_stats[2] = h[1];
        g_last_stats[3] = h[13]; g_last_stats[4] = h[14];
        fprintf(stderr, "t1dec stats: waves %u steps_total %llu symbols %llu max_steps %llu avg_steps/wave %.0f lane_eff %.3f events/wave %.0f"
                        " busiest lane %llu decisions in a wave of %llu steps\n",
                (nblocks + 63) / 64, h[0], h[1], h[2], (double)h[0] / ((nblocks + 63) / 64), (double)h[1] / (64.0 * h[0]),
                (double)h[3] / ((nblocks + 63) / 64), h[12] >> 32, h[12] & 0xffffffffull);
        if (nsolo) {
            const std::string tail = timing ? ", cycles/decision " + std::to_string((double)h[16] / (double)(h[13] ? h[13] : 1)) +
                                                  ", longest wave " + std::to_string(h[15] >> 20) + " cycles for " +
                                                  std::to_string(h[15] & 0xfffff) + " decisions"
                                            : std::string();
            fprintf(stderr, "t1dec solo: %u waves, decisions %llu, max per wave %llu%s\n", nsolo, h[13], h[14], tail.c_str());
        }
        if (timing)
            fprintf(stderr, "t1dec timing: cycles/event %.0f cycles/step %.0f (event share %.3f)\n",
                    (double)h[4] / (double)(h[3] ? h[3] : 1), (double)h[5] / (double)(h[0] ? h[0] : 1),
                    (double)h[4] / (double)(h[4] + h[5] ? h[4] + h[5] : 1));
        if (timing)
            fprintf(stderr, "t1dec event parts (max-lane sums / events): ring commit %.0f, write-back %.0f, select+LDS %.0f, "
                            "candidates %.0f, stage %.0f, prefetch %.0f\n",
                    (double)h[9] / (double)(h[3] ? h[3] : 1), (double)h[6] / (double)(h[3] ? h[3] : 1),
                    (double)h[7] / (double)(h[3] ? h[3] : 1), (double)h[8] / (double)(h[3] ? h[3] : 1),
                    (double)h[10] / (double)(h[3] ? h[3] : 1), (double)h[11] / (double)(h[3] ? h[3] : 1));
    }
}
void gk_launch_t1_recon(hipStream_t st, const GkBlock* blocks, const uint32_t* ids, const uint32_t* pos,
                        const uint64_t* scratch, const uint64_t* wave_off, int32_t* coef, uint32_t nblocks, uint32_t maxnp) {
    if (!nblocks) return;
    const uint32_t npmax = maxnp < 1 ? 1 : (maxnp > 32 ? 32 : maxnp);
    hipLaunchKernelGGL(k_t1_recon, dim3(nblocks), dim3(64), (size_t)(npmax + 1) * 64 * 8, st, blocks, ids, pos, scratch,
                       wave_off, coef, nblocks, npmax);
}
