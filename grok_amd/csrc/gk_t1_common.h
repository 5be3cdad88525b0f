// gk_t1_common.h — EBCOT/MQ tables and helpers shared by the T1 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// =============================================================================
// EBCOT context tables (ISO 15444-1 Annex D, Tables D.1-D.3), built in LDS at
// kernel start from the rules (no reference tables are copied).
//   zc index: 9-bit neighbourhood  bit0 NW bit1 N bit2 NE bit3 W bit4 (self) bit5 E bit6 SW bit7 S bit8 SE
//   sc index: 8-bit               bit0 W-neg bit1 W-sig bit2 E-neg bit3 E-sig bit4 N-neg bit5 N-sig bit6 S-neg bit7 S-sig
// =============================================================================
enum { CTX_ZC = 0, CTX_SC = 9, CTX_MAG = 14, CTX_AGG = 17, CTX_UNI = 18 };

// Lane conditions as VGPR masks (0 or 0xffffffff) combined with VALU logic and v_bfi selects.
// Measured on gfx950 with one wave per SIMD: a VALU compare feeding SALU mask logic (s_and_b64
// of lane masks) or a branch stalls the wave ~14-40 cycles per hop, a v_cndmask reading VCC can
// take ~14 cycles, while a VALU op issues every ~4.5 cycles; the decoder's step keeps its
// conditions in VGPRs.  opq() hides a value from the optimiser so it cannot turn the arithmetic
// back into compares on lane masks.
__device__ __forceinline__ uint32_t opq(uint32_t v) { asm volatile("" : "+v"(v)); return v; }
__device__ __forceinline__ uint32_t mbit(uint32_t v, uint32_t k) { return opq((uint32_t)__builtin_amdgcn_sbfe((int32_t)v, k, 1)); }
__device__ __forceinline__ uint32_t mneg(uint32_t v) { return mbit(v, 31); }   // sign -> mask
__device__ __forceinline__ uint32_t mlt(uint32_t a, uint32_t b) { return mneg(a - b); }   // a < b (|a - b| < 2^31)
__device__ __forceinline__ uint32_t mnz(uint32_t v) { return mneg(0u - v); }              // v != 0 (v < 2^31)
__device__ __forceinline__ uint32_t mz(uint32_t v) { return ~mnz(v); }                     // v == 0 (v < 2^31)

__device__ __forceinline__ uint32_t ffbh(uint32_t v) {   // leading zeros, 0xffffffff for 0
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(v));
    return r;
}
__device__ __forceinline__ uint32_t ffbl(uint32_t v) {   // lowest set bit, 0xffffffff for 0
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(v));
    return r;
}
// m ? a : b bitwise (v_bfi_b32 / v_bitop3_b32); m comes from the helpers above, so the optimiser
// cannot see it as a compare result and turn the select into a VCC select
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }


__host__ __device__ constexpr uint8_t zc_rule(uint32_t orient, uint32_t f) {
    int h = ((f >> 3) & 1) + ((f >> 5) & 1);
    int v = ((f >> 1) & 1) + ((f >> 7) & 1);
    int d = (f & 1) + ((f >> 2) & 1) + ((f >> 6) & 1) + ((f >> 8) & 1);
    if (orient == 1) { int t = h; h = v; v = t; }
    if (orient == 3) {
        int hv = h + v;
        if (d == 0) return hv == 0 ? 0 : (hv == 1 ? 1 : 2);
        if (d == 1) return hv == 0 ? 3 : (hv == 1 ? 4 : 5);
        if (d == 2) return hv == 0 ? 6 : 7;
        return 8;
    }
    if (h == 0) {
        if (v == 0) return d == 0 ? 0 : (d == 1 ? 1 : 2);
        return v == 1 ? 3 : 4;
    }
    if (h == 1) return v == 0 ? (d == 0 ? 5 : 6) : 7;
    return 8;
}
// returns (ctx offset in 0..4) | (xorbit << 4)
__host__ __device__ constexpr uint8_t sc_rule(uint32_t f) {
    auto c = [&](int sigbit, int negbit) { return ((f >> sigbit) & 1) ? (((f >> negbit) & 1) ? -1 : 1) : 0; };
    int H = c(1, 0) + c(3, 2), V = c(5, 4) + c(7, 6);
    H = H < -1 ? -1 : (H > 1 ? 1 : H);
    V = V < -1 ? -1 : (V > 1 ? 1 : V);
    if (H == 0 && V == 0) return 0;
    int xb = (H < 0 || (H == 0 && V < 0)) ? 1 : 0;
    if (H < 0) { H = -H; V = -V; }
    int ctx = (H == 0) ? 1 : (V == -1 ? 2 : (V == 0 ? 3 : 4));
    return (uint8_t)(ctx | (xb << 4));
}

// MQ probability estimation table (Annex C, Table C.2): qe | nmps<<16 | nlps<<22 | switch<<28
static __constant__ uint32_t c_mq[47] = {
    0x5601 | (1u << 16) | (1u << 22) | (1u << 28), 0x3401 | (2u << 16) | (6u << 22), 0x1801 | (3u << 16) | (9u << 22),
    0x0AC1 | (4u << 16) | (12u << 22), 0x0521 | (5u << 16) | (29u << 22), 0x0221 | (38u << 16) | (33u << 22),
    0x5601 | (7u << 16) | (6u << 22) | (1u << 28), 0x5401 | (8u << 16) | (14u << 22), 0x4801 | (9u << 16) | (14u << 22),
    0x3801 | (10u << 16) | (14u << 22), 0x3001 | (11u << 16) | (17u << 22), 0x2401 | (12u << 16) | (18u << 22),
    0x1C01 | (13u << 16) | (20u << 22), 0x1601 | (29u << 16) | (21u << 22), 0x5601 | (15u << 16) | (14u << 22) | (1u << 28),
    0x5401 | (16u << 16) | (14u << 22), 0x5101 | (17u << 16) | (15u << 22), 0x4801 | (18u << 16) | (16u << 22),
    0x3801 | (19u << 16) | (17u << 22), 0x3401 | (20u << 16) | (18u << 22), 0x3001 | (21u << 16) | (19u << 22),
    0x2801 | (22u << 16) | (19u << 22), 0x2401 | (23u << 16) | (20u << 22), 0x2201 | (24u << 16) | (21u << 22),
    0x1C01 | (25u << 16) | (22u << 22), 0x1801 | (26u << 16) | (23u << 22), 0x1601 | (27u << 16) | (24u << 22),
    0x1401 | (28u << 16) | (25u << 22), 0x1201 | (29u << 16) | (26u << 22), 0x1101 | (30u << 16) | (27u << 22),
    0x0AC1 | (31u << 16) | (28u << 22), 0x09C1 | (32u << 16) | (29u << 22), 0x08A1 | (33u << 16) | (30u << 22),
    0x0521 | (34u << 16) | (31u << 22), 0x0441 | (35u << 16) | (32u << 22), 0x02A1 | (36u << 16) | (33u << 22),
    0x0221 | (37u << 16) | (34u << 22), 0x0141 | (38u << 16) | (35u << 22), 0x0111 | (39u << 16) | (36u << 22),
    0x0085 | (40u << 16) | (37u << 22), 0x0049 | (41u << 16) | (38u << 22), 0x0025 | (42u << 16) | (39u << 22),
    0x0015 | (43u << 16) | (40u << 22), 0x0009 | (44u << 16) | (41u << 22), 0x0005 | (45u << 16) | (42u << 22),
    0x0001 | (45u << 16) | (43u << 22), 0x5601 | (46u << 16) | (46u << 22)};

// The hot coders keep a context as the entry of its (state, MPS) pair: entry 2 s + m =
// Qe | (2 NMPS + m) << 16 | (2 NLPS + (m ^ SWITCH)) << 23 | m << 31, so both successor entries,
// MPS bit included, are one table read away and no MPS arithmetic follows the decision (94
// entries; the initial states of mqc_resetstates are entries 2 s).
#define MQ_PAIRS 94
__device__ __forceinline__ uint32_t mq_pair_entry(uint32_t j) {
    const uint32_t e = c_mq[j >> 1], m = j & 1;
    return (e & 0xffffu) | ((2 * ((e >> 16) & 0x3f) + m) << 16) | ((2 * ((e >> 22) & 0x3f) + (m ^ ((e >> 28) & 1))) << 23) |
           (m << 31);
}

