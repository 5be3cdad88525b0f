// gk_t1enc.hip — parallel Part-1 T1 encoder for CDNA4 (two kernels).
//
//  k_t1_cm  (one wave per code-block, lane = column): EBCOT context modelling.
//           All three coding passes (T1.cpp:498-780) are evaluated for a whole
//           4-row stripe at once with 64-bit column masks.  The only causal
//           chain — significance propagation spreading left->right inside a
//           stripe — is solved by a wave-wide fixpoint (monotone, converges to
//           the sequential result); everything else is data-parallel because
//           the encoder knows every magnitude bit up front.  Each stripe-pass
//           emits its (context, decision) symbols in scan order through a wave
//           prefix sum into a per-block symbol stream.
//  k_t1_mq  (one lane per code-block): the MQ arithmetic coder (Annex C;
//           mqc_enc.cpp:86-330) over that symbol stream, plus Grok's pass
//           bookkeeping (rates, termination, monotone fix, FF back-off;
//           T1.cpp:856-930).
//
// Symbol byte = (ctx << 1) | decision, ctx in 0..18 (T1_CTXNO_*).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"
#include "gk_t1_common.h"
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#define SYM_PER_PLANE 11264u   // >= 2 symbols per sample + 3 per stripe column, per bit-plane

__device__ __forceinline__ uint32_t win6(uint64_t col, uint32_t s) {
    return (uint32_t)((s ? (col >> (4 * s - 1)) : (col << 1)) & 63u);
}

// Cross-lane moves through DPP (a few cycles) instead of LDS permutes (~50-cycle round trips,
// which made the modelling of a stripe a chain of dependent LDS latencies).
__device__ __forceinline__ uint32_t lane_prev(uint32_t v) {   // lane - 1's value, 0 at lane 0 (wave_shr:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t lane_next(uint32_t v) {   // lane + 1's value, 0 at lane 63 (wave_shl:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}
// exclusive prefix sum over the wave (row_shr 1/2/4/8 within rows of 16, then row_bcast 15 / 31)
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
    int inc = (int)v;
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x111, 0xf, 0xf, false);
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x112, 0xf, 0xf, false);
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x114, 0xf, 0xf, false);
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x118, 0xf, 0xf, false);
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x142, 0xa, 0xf, false);
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x143, 0xc, 0xf, false);
    total = (uint32_t)__builtin_amdgcn_readlane(inc, 63);
    return (uint32_t)inc - v;
}

// 3x3 neighbourhood of stripe row r in column-major order: bits 0-2 the left column, 3-5 the
// centre, 6-8 the right one, each as rows r-1, r, r+1 (6-bit column windows: bit0 = the row above
// the stripe, bit5 = the row below, so row r - 1 + k is window bit r + k).  Three bit-field
// extracts per row instead of nine single-bit moves; the context tables are built in this order.
__device__ __forceinline__ uint32_t nb9(uint32_t L, uint32_t C, uint32_t R, int r) {
    return ((L >> r) & 7u) | (((C >> r) & 7u) << 3) | (((R >> r) & 7u) << 6);
}
// sign-context index from the significance (fs) and sign (fn) neighbourhoods of nb9:
// bit0 W-neg bit1 W-sig bit2 N-neg bit3 N-sig bit4 S-neg bit5 S-sig bit6 E-neg bit7 E-sig
__device__ __forceinline__ uint32_t sc8(uint32_t fs, uint32_t fn) { return (fs & 0xaau) | ((fn >> 1) & 0x55u); }
// table index -> the rule functions' layouts (gk_t1_common.h)
__host__ __device__ constexpr uint32_t zc_of_nb9(uint32_t i) {
    return (i & 1u) | (((i >> 3) & 1u) << 1) | (((i >> 6) & 1u) << 2) | (((i >> 1) & 1u) << 3) | (((i >> 4) & 1u) << 4) |
           (((i >> 7) & 1u) << 5) | (((i >> 2) & 1u) << 6) | (((i >> 5) & 1u) << 7) | (((i >> 8) & 1u) << 8);
}
__host__ __device__ constexpr uint32_t sc_of_sc8(uint32_t i) {
    return (i & 3u) | (((i >> 6) & 3u) << 2) | (((i >> 2) & 3u) << 4) | (((i >> 4) & 3u) << 6);
}
// The context tables in nb9 / sc8 order, evaluated at compile time (a block's wave copies its
// orientation's 768 bytes into LDS instead of evaluating the rules for 768 entries).
struct alignas(16) CmTabs {
    uint8_t zc[4][512];
    uint8_t sc[256];
};
constexpr CmTabs make_cm_tabs() {
    CmTabs t{};
    for (uint32_t o = 0; o < 4; ++o)
        for (uint32_t i = 0; i < 512; ++i) t.zc[o][i] = zc_rule(o, zc_of_nb9(i));
    for (uint32_t i = 0; i < 256; ++i) t.sc[i] = sc_rule(sc_of_sc8(i));
    return t;
}
__constant__ CmTabs c_cm_tabs = make_cm_tabs();

struct alignas(16) CmLds {
    uint8_t zc[512];
    uint8_t sc[256];
};
// Rate-control extras: the nmsedec tables (t1_generate_luts.cpp:338-362: sig, sig0, ref,
// ref0; 128 entries each, built on the host).  The magnitudes the lookups index stay in the
// lane's registers: a pass's samples are summed after it from a 64-row mask.
struct CmRcLds {
    int16_t nm[4][128];
};

__device__ __forceinline__ int32_t wave_sum(int32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// RC: also accumulate Grok's per-pass nmsedec (T1.cpp:483-764 getnmsedec_sig/_ref)
// into pass_nmse[b * GK_MAX_PASSES + pass].
template <bool RC>
__global__ __launch_bounds__(64) void k_t1_cm(const int32_t* __restrict__ coef, const GkBlock* __restrict__ blocks,
                                              const uint64_t* __restrict__ sym_off, uint8_t* __restrict__ sym,
                                              uint32_t* __restrict__ pass_end, uint32_t* __restrict__ cm_info,
                                              uint32_t nblocks, int* err, const int16_t* __restrict__ nmse_tab,
                                              int32_t* __restrict__ pass_nmse, const uint32_t* __restrict__ order,
                                              uint32_t base, uint32_t count) {
    __shared__ CmLds L;
    __shared__ typename std::conditional<RC, CmRcLds, char>::type R;
    // workgroup j codes block order[base + j] (all blocks in index order without an order)
    if (blockIdx.x >= count) return;
    const uint32_t b = order ? order[base + blockIdx.x] : base + blockIdx.x;
    if (b >= nblocks) return;
    const int lane = threadIdx.x;
    const GkBlock B = blocks[b];
    const uint32_t w = B.w, h = B.h;
    reinterpret_cast<uint2*>(L.zc)[lane] = reinterpret_cast<const uint2*>(c_cm_tabs.zc[B.orient & 3])[lane];
    reinterpret_cast<uint32_t*>(L.sc)[lane] = reinterpret_cast<const uint32_t*>(c_cm_tabs.sc)[lane];
    // ---- quantise + sign-magnitude (T1Part1.cpp:36-87), column `lane` into registers
    const bool irrev = B.flags & 1;
    uint32_t m[64];
    uint64_t negcol = 0;
    uint32_t mx = 0;
#pragma unroll
    for (int y = 0; y < 64; ++y) {
        int32_t v = 0;
        if (y < (int)h && lane < (int)w) {
            int32_t raw = coef[B.band_off + (size_t)y * B.stride + lane];
            if (irrev) v = (int32_t)rintf((__int_as_float(raw) / B.step) * 64.0f);
            else v = raw * 64;
        }
        uint32_t a = (uint32_t)(v < 0 ? -v : v);
        m[y] = a;
        mx = a > mx ? a : mx;
        negcol |= (uint64_t)(v < 0) << y;
    }
    if (const uint32_t rs = B.flags >> 3) {   // ROI maxshift (the component is the region): index integer part up
        mx = 0;
#pragma unroll
        for (int y = 0; y < 64; ++y) {
            m[y] = ((m[y] >> 6) << (6 + rs)) | (m[y] & 63u);
            mx = m[y] > mx ? m[y] : mx;
        }
    }
    if constexpr (RC) {
        for (int i = lane; i < 512; i += 64) R.nm[i >> 7][i & 127] = nmse_tab[i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { uint32_t t = __shfl_xor(mx, o); mx = t > mx ? t : mx; }
    uint32_t numbps = 0;
    if (mx) { uint32_t t = 32 - __clz(mx); numbps = t <= 6 ? 0 : t - 6; }
    __syncthreads();
    if (numbps == 0) {
        if (lane == 0) { cm_info[2 * b] = 0; cm_info[2 * b + 1] = 0; }
        return;
    }
    const uint64_t base_off = sym_off[b];
    const uint64_t cap = sym_off[b + 1] - base_off;
    if ((uint64_t)numbps * SYM_PER_PLANE > cap) {
        if (lane == 0) { atomicOr(err, 2); cm_info[2 * b] = 0; cm_info[2 * b + 1] = 0; }
        return;
    }
    uint8_t* S = sym + base_off;
    uint32_t* PE = pass_end + (size_t)b * GK_MAX_PASSES;
    const uint64_t validcol = (lane < (int)w) ? ((h >= 64) ? ~0ull : ((1ull << h) - 1)) : 0ull;
    const uint32_t nstripes = (h + 3) >> 2;
    uint64_t sig = 0, mu = 0;
    uint32_t pos = 0, passno = 0;
    int32_t acc = 0;   // RC: this lane's nmsedec for the current pass
    // RC: nmsedec of the rows in mask (getnmsedec_sig: table 0/1, getnmsedec_ref: table 2/3)
    // (8-row groups that no lane of the wave has in `mask` are skipped with one uniform branch:
    // a pass's new significances are sparse at the upper planes)
    auto nm_rows = [&](uint64_t mask, int t, int bp) __attribute__((always_inline)) {
        if constexpr (RC) {
            const int16_t* tab = R.nm[bp > 0 ? t : t + 1];
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const uint32_t gm = (uint32_t)(mask >> (8 * g)) & 0xffu;
                if (__any(gm != 0)) {
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if ((gm >> k) & 1) acc += tab[(m[8 * g + k] >> bp) & 127];
                }
            }
        }
    };
    auto end_pass = [&]() {
        if (lane == 0) PE[passno] = pos;
        if constexpr (RC) {
            int32_t t = wave_sum(acc);
            if (lane == 0) pass_nmse[(size_t)b * GK_MAX_PASSES + passno] = t;
            acc = 0;
        }
        ++passno;
    };

    for (int bpno = (int)numbps - 1; bpno >= 0; --bpno) {
        uint64_t bitcol = 0;
#pragma unroll
        for (int y = 0; y < 64; ++y) bitcol |= (uint64_t)((m[y] >> (bpno + 6)) & 1u) << y;
        uint64_t vis = 0;
        const uint64_t sigPrev = sig;
        if (bpno != (int)numbps - 1) {
            // ================= significance propagation pass =================
            for (uint32_t s = 0; s < nstripes; ++s) {
                const uint32_t sh = 4 * s;
                const uint32_t Wc = win6(sig, s), Nc = win6(negcol, s);
                uint32_t pk = Wc | (Nc << 6);
                const uint32_t pL = lane_prev(pk), pR = lane_next(pk);
                const uint32_t WL = pL & 63, NL = (pL >> 6) & 63, WR = pR & 63, NR = (pR >> 6) & 63;
                const uint32_t valid4 = (uint32_t)(validcol >> sh) & 15u;
                const uint32_t cand = ~(Wc >> 1) & valid4;
                const uint32_t bit4 = (uint32_t)(bitcol >> sh) & 15u;
                const uint32_t A = ((WL | (WL >> 1) | (WL >> 2)) | (WR | (WR >> 1) | (WR >> 2)) | Wc | (Wc >> 2)) & 15u;
                auto F = [&](uint32_t in, uint32_t& cd) -> uint32_t {
                    uint32_t x = A | ((in | (in << 1) | (in >> 1)) & 15u);
                    uint32_t c0 = cand & x & 1u, n0 = c0 & bit4;
                    uint32_t c1 = cand & (x | (n0 << 1)) & 2u, n1 = c1 & bit4;
                    uint32_t c2 = cand & (x | (n1 << 1)) & 4u, n2 = c2 & bit4;
                    uint32_t c3 = cand & (x | (n2 << 1)) & 8u, n3 = c3 & bit4;
                    cd = c0 | c1 | c2 | c3;
                    return n0 | n1 | n2 | n3;
                };
                uint32_t cd, in = 0;
                uint32_t ns = F(0, cd);
                while (true) {
                    in = lane_prev(ns);
                    uint32_t cd2, ns2 = F(in, cd2);
                    bool ch = ns2 != ns;
                    ns = ns2; cd = cd2;
                    if (!__any(ch)) break;
                }
                // symbols.  The left column is coded before this one (its new significances count),
                // the right one after; in this column the rows above r are coded before row r.
                const uint32_t Lt = WL | (in << 1), Cn = ns << 1;
                uint32_t cnt = __popc(cd) + __popc(ns);
                uint32_t total, off = wave_excl_scan(cnt, total);
                uint8_t* o = S + pos + off;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if ((cd >> r) & 1) {
                        const uint32_t d = (bit4 >> r) & 1;
                        const uint32_t fs = nb9(Lt, Wc | (Cn & ((2u << r) - 1)), WR, r);
                        *o++ = (uint8_t)(((CTX_ZC + L.zc[fs]) << 1) | d);
                        if (d) {
                            const uint32_t e = L.sc[sc8(fs, nb9(NL, Nc, NR, r))];
                            const uint32_t sg = (Nc >> (r + 1)) & 1;
                            *o++ = (uint8_t)(((CTX_SC + (e & 15)) << 1) | (sg ^ (e >> 4)));
                        }
                    }
                }
                pos += total;
                sig |= (uint64_t)ns << sh;
                vis |= (uint64_t)cd << sh;
            }
            nm_rows(sig & ~sigPrev, 0, bpno);
            end_pass();
            // ================= magnitude refinement pass =================
            for (uint32_t s = 0; s < nstripes; ++s) {
                const uint32_t sh = 4 * s;
                const uint32_t Wc = win6(sig, s);
                const uint32_t pL = lane_prev(Wc), pR = lane_next(Wc);
                const uint32_t nb = ((pL | (pL >> 1) | (pL >> 2)) | (pR | (pR >> 1) | (pR >> 2)) | Wc | (Wc >> 2)) & 15u;
                const uint32_t mr = (uint32_t)(sigPrev >> sh) & 15u;
                const uint32_t mu4 = (uint32_t)(mu >> sh) & 15u;
                const uint32_t bit4 = (uint32_t)(bitcol >> sh) & 15u;
                uint32_t total, off = wave_excl_scan(__popc(mr), total);
                uint8_t* o = S + pos + off;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if ((mr >> r) & 1) {
                        uint32_t cx = ((mu4 >> r) & 1) ? CTX_MAG + 2 : (((nb >> r) & 1) ? CTX_MAG + 1 : CTX_MAG);
                        *o++ = (uint8_t)((cx << 1) | ((bit4 >> r) & 1));
                    }
                }
                pos += total;
            }
            nm_rows(sigPrev, 2, bpno);
            mu |= sigPrev;
            end_pass();
        }
        // ================= cleanup pass =================
        const uint64_t sigCu = sig;
        for (uint32_t s = 0; s < nstripes; ++s) {
            const uint32_t sh = 4 * s;
            const uint32_t Wc = win6(sig, s), Nc = win6(negcol, s);
            const uint32_t valid4 = (uint32_t)(validcol >> sh) & 15u;
            const uint32_t vis4 = (uint32_t)(vis >> sh) & 15u;
            const uint32_t bit4 = (uint32_t)(bitcol >> sh) & 15u;
            const uint32_t cl = ~(Wc >> 1) & ~vis4 & valid4;
            const uint32_t nc = cl & bit4;
            uint32_t pk = Wc | (Nc << 6) | (nc << 12);
            const uint32_t pL = lane_prev(pk), pR = lane_next(pk);
            const uint32_t WL = pL & 63, NL = (pL >> 6) & 63, ncL = (pL >> 12) & 15;
            const uint32_t WR = pR & 63, NR = (pR >> 6) & 63;
            const uint32_t Lt = WL | (ncL << 1), Cn = nc << 1;
            const bool agg = (valid4 == 15u) && (cl == 15u) && ((Lt | WR | (Wc & 0x21u)) == 0);
            uint32_t rl = nc ? (uint32_t)__ffs(nc) - 1 : 4u;
            uint32_t cnt;
            uint32_t codemask;   // rows coded with ZC
            if (agg) {
                if (rl == 4) { cnt = 1; codemask = 0; }
                else {
                    codemask = cl & ~((2u << rl) - 1);   // rows after the run
                    cnt = 3 + 1 + __popc(codemask) + __popc(nc & codemask);
                }
            } else {
                codemask = cl;
                cnt = __popc(cl) + __popc(nc);
            }
            uint32_t total, off = wave_excl_scan(cnt, total);
            uint8_t* o = S + pos + off;
            if (agg) {
                *o++ = (uint8_t)((CTX_AGG << 1) | (rl != 4 ? 1 : 0));
                if (rl != 4) {
                    *o++ = (uint8_t)((CTX_UNI << 1) | (rl >> 1));
                    *o++ = (uint8_t)((CTX_UNI << 1) | (rl & 1));
                    // the run's column and its neighbours are insignificant, and so are the rows the
                    // run covered: the sign context of an empty neighbourhood (CTX_SC, no flip)
                    const uint32_t sg = (Nc >> (rl + 1)) & 1;
                    *o++ = (uint8_t)((CTX_SC << 1) | sg);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if ((codemask >> r) & 1) {
                    const uint32_t d = (bit4 >> r) & 1;
                    const uint32_t fs = nb9(Lt, Wc | (Cn & ((2u << r) - 1)), WR, r);
                    *o++ = (uint8_t)(((CTX_ZC + L.zc[fs]) << 1) | d);
                    if (d) {
                        const uint32_t e = L.sc[sc8(fs, nb9(NL, Nc, NR, r))];
                        const uint32_t sg = (Nc >> (r + 1)) & 1;
                        *o++ = (uint8_t)(((CTX_SC + (e & 15)) << 1) | (sg ^ (e >> 4)));
                    }
                }
            }
            pos += total;
            sig |= (uint64_t)nc << sh;
        }
        nm_rows(sig & ~sigCu, 0, bpno);
        end_pass();
    }
    if (lane == 0) { cm_info[2 * b] = numbps; cm_info[2 * b + 1] = passno; }
}

// ---------------------------------------------------------------------------
// MQ coder (Annex C.2; mqc_enc.cpp:86-330), one lane per code-block.
// Every lane codes exactly one symbol per step, so all lanes of a wave sit at
// the same symbol index: the 16-symbol chunks of every lane are fetched at the
// same (uniform) steps, two chunks ahead, and the loop is unrolled by 16 so a
// fetch is consumed 32 steps after it was issued.  Pass boundaries come from a
// per-lane copy of the pass-end table in LDS.
// Context states live in LDS per lane as their probability-table entry with the
// MPS in bit 31 (one read gives Qe, NMPS, NLPS and SWITCH; the next entry is
// written back off the symbol's dependency chain), as in the decoder.
// Output bytes gather into dwords in a VGPR; every emission stores the dword it touched into a
// per-lane 128-byte ring (two 64-byte lines) in LDS, unconditionally (a later store of the same
// dword supersedes it), and a completed line leaves as four 16-byte stores at the next 16-symbol
// group boundary (a symbol emits at most two bytes, so a group crosses at most one line end), so
// HBM sees whole lines instead of one 4-byte write per lane-dword (scattered over 64 slots).
// Lane conditions are 0 / -1 VGPR values combined with VALU logic (gk_t1_common.h), not compare
// masks in SGPRs: a compare feeding SALU mask logic stalls a lone wave ~14 cycles per hop.
// ---------------------------------------------------------------------------
#define MQ_RING_DW 32
struct MqLane {
    uint32_t a, c, ct;
    int32_t bp;
    uint32_t cur;
    uint8_t* out;
    uint32_t cap;
    uint32_t lf;             // first line of the stream not yet stored to HBM
    // context-state update of the last symbol, not yet in LDS (cx 19 = none), and the entry of
    // the next symbol's context read ahead of time (see mq_code5)
    uint32_t pcx1, pne1, epref;
};
struct MqLds {
    uint32_t tab[96];                     // (state, MPS) pair entries (mq_pair_entry)
    uint32_t ctx[20][64];                 // per-lane context states (table entry | MPS << 31); row 19 spare
    uint32_t ring[64][MQ_RING_DW + 1];    // per-lane output ring (row padded: conflict-free columns)
};

// stream line `li` (64 bytes from the lane's ring) to HBM; only whole lines inside the slot
__device__ __forceinline__ void mq_line_store(MqLane& q, MqLds& L, int lane, uint32_t li) {
    const uint32_t o = (li & 1) * 16;
    uint8_t* dst = q.out + (size_t)li * 64;
    if ((li + 1) * 64 <= q.cap) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *(uint4*)(dst + 16 * i) = make_uint4(L.ring[lane][o + 4 * i], L.ring[lane][o + 4 * i + 1],
                                                 L.ring[lane][o + 4 * i + 2], L.ring[lane][o + 4 * i + 3]);
    } else {
        for (uint32_t i = 0; i < 16 && li * 64 + 4 * i + 4 <= q.cap; ++i) *(uint32_t*)(dst + 4 * i) = L.ring[lane][o + i];
    }
}
// the lines the stream has passed (at most one per 16-symbol group) go out
__device__ __forceinline__ void mq_lines_out(MqLane& q, MqLds& L, int lane) {
    const uint32_t cl = (uint32_t)max(q.bp, 0) >> 6;
    if (__any(cl > q.lf)) {
        if (cl > q.lf) { mq_line_store(q, L, lane, q.lf); q.lf++; }
    }
}

// byte `cur` to stream position bp where bo (a lane mask), bp advances.  The byte is stored into
// the lane's ring unconditionally (one ds_write_b8): where bo is clear it lands at bp, past the
// stream, and the lane's next byte overwrites it before its line goes out.  The coder's dummy
// byte at bp = -1 lands in ring byte 127, rewritten by stream byte 127 before line 1 leaves;
// bytes at or past cap enter the ring but never HBM (line stores stop at cap; the final bp
// reports the overflow).
__device__ __forceinline__ void mq_put5(MqLane& q, MqLds& L, int lane, uint32_t bo, uint32_t cur) {
    uint8_t* row = reinterpret_cast<uint8_t*>(&L.ring[lane][0]);
    row[(uint32_t)q.bp & (4 * MQ_RING_DW - 1)] = (uint8_t)cur;
    q.bp -= (int32_t)bo;
}
// BYTEOUT (Annex C.2.6, mqc_enc.cpp:86-127) where bo (a lane mask; CT has reached 0 there).
// The finished byte (cur plus the carry) goes to position bp: into the dword buffer and,
// unconditionally, into the ring (bp = -1 is the coder's dummy byte before the buffer, and
// bytes at or past cap are dropped: the final bp reports the overflow).
// CARRY = false: C is known to be below 2^27 (a second BYTEOUT in one renormalisation: the first
// left C below 2^20 and at most 8 shifts followed), so the carry test is left out.
template <bool CARRY = true>
__device__ __forceinline__ void mq_byteout5(MqLane& q, MqLds& L, int lane, uint32_t bo, uint32_t& c, uint32_t& ct) {
    uint32_t cur = q.cur;
    if constexpr (CARRY) {
        const uint32_t carry = (c >> 27) & 1u & bo & ~mz(q.cur ^ 0xffu);
        cur += carry;
        c &= ~(carry << 27);
    }
    const uint32_t ffm = mz(cur ^ 0xffu);                          // 0 / -1
    const uint32_t nb = __builtin_amdgcn_ubfe(c, 19u - ffm, 8);    // C >> 20 after 0xFF, else C >> 19
    mq_put5(q, L, lane, bo, cur);
    q.cur = bsel(bo, nb, q.cur);
    c &= (0x7ffffu | (ffm & 0x80000u)) | ~bo;
    ct = bsel(bo, 8u + ffm, ct);                                    // 7 after 0xFF, else 8
}

// CODEMPS / CODELPS + RENORME (Annex C.2.4-C.2.7), branch-free.  With x = (MPS symbol) xor
// (A - Qe < Qe): the coder adds Qe to C iff x and keeps A - Qe iff x, else A = Qe.
// RENORME's n = clz shifts run as at most three straight shifts: up to the byte boundary
// (CT = 0), BYTEOUT there, then the rest; C stays below 2^28 before a shift of at most CT, so
// 32 bits hold it.  A second boundary needs n >= CT + 7 (rare; never a third for n <= 15).
// One symbol (cx = s >> 1, decision s & 1).  A lane past its block's last symbol keeps coding
// (zero bytes: context 0, decision 0) with CT parked at 2^30 by its flush, so it never reaches a
// BYTEOUT again and its stream position, pending byte and lines stay as the flush left them; A
// stays a valid interval for any symbol, so no per-symbol "lane has a symbol" mask is needed.
// Context states reach LDS one symbol late: the entry of the next symbol's context is read
// here, right after the previous symbol's update is written, and the next symbol takes this
// symbol's update from registers when its context matches.  So neither the context read nor
// the probability-table read of an update sits on the chain between consecutive symbols
// (except for back-to-back symbols of one context, which wait for the table read).
#define MQ_CT_PARKED (1u << 30)
__device__ __forceinline__ void mq_code5(MqLane& q, MqLds& L, int lane, uint32_t s, uint32_t s_next) {
    // bytes past a block's symbols are arbitrary: their context is the spare row 19
    const uint32_t cx = min(s >> 1, 19u);
    // (opq on the operands: the optimiser would turn the equality masks back into compares)
    const uint32_t e = bsel(mz(opq(cx ^ q.pcx1)), q.pne1, q.epref);
    L.ctx[q.pcx1][lane] = q.pne1;                         // the previous symbol's update
    q.epref = L.ctx[min(s_next >> 1, 19u)][lane];
    const uint32_t mpsm = mneg(e), qe = e & 0xffff;
    const uint32_t a1 = q.a - qe;
    const uint32_t ism = ~(mpsm ^ mbit(s, 0));            // the symbol is the MPS
    const uint32_t fast = ism & mbit(a1, 15);             // MPS without renormalisation
    const uint32_t x = ism ^ mlt(a1, qe);
    // the successor pair entry (MPS bit included): NMPS for the MPS, NLPS (with SWITCH) for the LPS
    uint32_t nidx;   // one v_bfi (the compiler otherwise masks both fields and adds them scaled)
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(nidx) : "v"(ism), "v"(__builtin_amdgcn_ubfe(e, 16, 7)), "v"(__builtin_amdgcn_ubfe(e, 23, 7)));
    const uint32_t ne = L.tab[nidx];
    q.pcx1 = cx; q.pne1 = bsel(fast, e, ne);
    const uint32_t an = bsel(x, a1, qe);
    const uint32_t n = ffbh(an) - 16u;                    // an != 0; 0 on the fast path (an = a1 >= 0x8000)
    q.a = an << n;
    uint32_t c = q.c + (qe & x);
    const uint32_t n1 = min(n, q.ct);
    uint32_t n2 = n - n1;
    const bool two = __any(n2 >= 7u);                      // known before the first BYTEOUT
    c <<= n1;
    uint32_t ct = q.ct - n1;
    mq_byteout5(q, L, lane, mz(ct), c, ct);
    if (two) {
        const uint32_t n2a = min(n2, ct);
        c <<= n2a; ct -= n2a; n2 -= n2a;
        mq_byteout5<false>(q, L, lane, mz(ct), c, ct);
    }
    q.c = c << n2;
    q.ct = ct - n2;
}

__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t j) {
    const uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
    return (w >> (8 * (j & 3))) & 0xff;
}

// ------------------------------------------------------------------ solo MQ coding
// The heaviest blocks set the lane-parallel kernel's time: a lane codes one symbol per ~440
// cycles whatever its own path (every lane runs every select of the step), and the LL and
// low-resolution blocks of C3's 12-bit 9/7 data carry ~65 k symbols against a ~37 k plateau.
// Solo waves code one such block each with the coder wave-uniform: A, C, CT and the byte
// position in SGPRs, SALU selects instead of lane masks, the context states in lanes 0..18 of a
// VGPR and the (state, MPS) pair table in two VGPRs (v_readlane / v_writelane), the symbols
// arriving 64 at a time as 16 dwords in lanes 0..15, finished bytes gathered into a dword that
// lane 0 stores.  The coder is the standard one of Annex C.2 in Grok's 32-bit arithmetic
// (mqc_enc.cpp:86-330: C with its carry at bit 27, as gk_t1ms.hip's MsEnc), the pass bookkeeping
// k_t1_mq's (T1.cpp:856-930); outputs are the same records, so T2 and rate control are shared.
__device__ __forceinline__ uint32_t srl(uint32_t v, uint32_t lane) {   // v_readlane_b32
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}
__device__ __forceinline__ uint32_t swl(uint32_t old, uint32_t val, uint32_t lane) {   // v_writelane_b32
    // (gfx9 reads one SGPR per VALU op besides M0: the lane select goes through M0)
    asm("v_writelane_b32 %0, %1, m0" : "+v"(old) : "s"(val), "{m0}"(lane));
    return old;
}
// Output: finished bytes gather into a dword (wacc, SGPR) written into a 256-byte ring held as one
// VGPR (lane k = ring dword k) with v_writelane after every byte; at the end of every 64-symbol
// chunk the 64-byte lines the stream has passed leave as one 16-lane store each (a chunk emits at
// most 128 bytes).  No divergent branch sits in the symbol loop.
struct MqSolo {
    uint32_t a, c, ct;
    int32_t bp;          // position of the pending byte `cur` (-1: the coder's dummy byte)
    uint32_t cur;
    uint32_t wacc;       // finished bytes of the dword holding position bp
    uint32_t ring;       // (VGPR) 256-byte ring of the stream, lane k = dword k
    // BYTEOUT (mqc_byteout, mqc_enc.cpp:86-127) without branches: a carry (C bit 27, unless the
    // pending byte is 0xFF) goes into the pending byte, which is then final; the next byte takes 7
    // bits of C after an 0xFF, else 8
    __device__ __forceinline__ void byteout() {
        const bool ff = cur == 0xffu;
        const bool carry = !ff && (c & 0x8000000u);
        const uint32_t cur2 = cur + (carry ? 1u : 0u);
        const bool seven = cur2 == 0xffu;
        const uint32_t cc = carry ? c & 0x7ffffffu : c;
        const uint32_t nb = seven ? (cc >> 20) & 0xffu : (cc >> 19) & 0xffu;
        // cur2 is final at bp (bp = -1: the dummy byte lands in ring dword 63, rewritten by stream
        // bytes 252..255 before that line leaves)
        wacc |= cur2 << (8u * ((uint32_t)bp & 3u));
        ring = swl(ring, wacc, ((uint32_t)bp >> 2) & 63u);
        ++bp;
        wacc = ((uint32_t)bp & 3u) ? wacc : 0u;
        cur = nb;
        c = seven ? cc & 0xfffffu : cc & 0x7ffffu;
        ct = seven ? 7u : 8u;
    }
};

__device__ void mq_solo_block(uint32_t b, const uint8_t* __restrict__ sym, const uint64_t* __restrict__ sym_off,
                              const uint32_t* __restrict__ pass_end, const uint32_t* __restrict__ cm_info,
                              const GkBlock* __restrict__ blocks, uint8_t* __restrict__ bytes,
                              GkPass* __restrict__ passes, uint32_t* __restrict__ info, int* err,
                              const int32_t* __restrict__ pass_nmse, uint32_t* __restrict__ pass_counter, int lane) {
    const uint32_t numbps = cm_info[2 * b], npasses = cm_info[2 * b + 1];
    if (npasses == 0) {
        if (lane == 0) { info[4 * b] = 0; info[4 * b + 1] = 0; info[4 * b + 2] = 0; info[4 * b + 3] = 0; }
        return;
    }
    const uint32_t* PE = pass_end + (size_t)b * GK_MAX_PASSES;
    const uint32_t nsym = PE[npasses - 1];
    const GkBlock B = blocks[b];
    const uint8_t* sp = sym + sym_off[b];
    uint8_t* out = bytes + B.data_off;
    const uint32_t cap = B.data_cap;
    uint32_t poff = 0;
    if (lane == 0) poff = atomicAdd(pass_counter, npasses);
    poff = srl(poff, 0);
    GkPass* P = passes + poff;
    const bool rc = (B.flags & 2) != 0;
    double cum = 0.0;
    // the pair table and the context states in lanes (mqc_resetstates: ZC0 = 4, AGG = 3, UNI = 46)
    const uint32_t TAB0 = mq_pair_entry((uint32_t)lane), TAB1 = lane < MQ_PAIRS - 64 ? mq_pair_entry(64u + lane) : 0u;
    uint32_t CTX = mq_pair_entry(2u * (lane == CTX_ZC ? 4u : (lane == CTX_AGG ? 3u : (lane == CTX_UNI ? 46u : 0u))));
    MqSolo q;
    q.a = 0x8000; q.c = 0; q.ct = 12; q.bp = -1; q.cur = 0; q.wacc = 0; q.ring = 0;
    uint32_t lf = 0;   // first 64-byte line not yet stored
    auto lines_out = [&](uint32_t upto) {   // lines [lf, upto) from the ring, 16 lanes each
        for (; lf < upto; ++lf)
            if ((uint32_t)(lane >> 4) == (lf & 3u) && lf * 64 + 64 <= cap)
                *reinterpret_cast<uint32_t*>(out + (size_t)lf * 64 + 4 * (lane & 15)) = q.ring;
    };
    auto chunk = [&](uint32_t k) -> uint32_t {   // symbols [64 k, 64 k + 64) as dwords in lanes 0..15
        return (lane < 16 && 64 * k < nsym) ? *reinterpret_cast<const uint32_t*>(sp + 64 * k + 4 * lane) : 0u;
    };
    uint32_t p = 0, next_end = PE[0];
    auto close_pass = [&]() {   // pass p ends here (T1.cpp:856-897)
        uint32_t rate;
        if (p == npasses - 1) {   // FLUSH (mqc_enc.cpp:213-227); the last pass is the one terminated
            const uint32_t tempc = q.c + q.a;
            q.c |= 0xffffu;
            if (q.c >= tempc) q.c -= 0x8000u;
            q.c <<= q.ct; q.byteout();
            q.c <<= q.ct; q.byteout();
            // a final 0xFF is not part of the stream; any other pending byte is
            if (q.cur != 0xffu) {
                q.wacc |= q.cur << (8u * ((uint32_t)q.bp & 3u));
                q.ring = swl(q.ring, q.wacc, ((uint32_t)q.bp >> 2) & 63u);
                ++q.bp;
            }
            rate = (uint32_t)q.bp;
        } else {
            rate = (uint32_t)q.bp + 5u + (q.ct < 5 ? 1u : 0u);
        }
        if (rc) {
            const int bpno = p == 0 ? (int)numbps - 1 : (int)numbps - 2 - (int)(p - 1) / 3;
            double wm = __dmul_rn(B.wmse, (double)(1 << bpno));
            wm = __dmul_rn(wm, __dmul_rn(wm, (double)pass_nmse[(size_t)b * GK_MAX_PASSES + p]) / 8192.0);
            cum = __dadd_rn(cum, wm);
        }
        if (lane == 0) { P[p].rate = rate; P[p].dist = cum; }
        ++p;
        next_end = p < npasses ? PE[p] : 0xffffffffu;
    };
    while (p < npasses && next_end == 0) close_pass();   // passes without symbols
    uint32_t NX = chunk(0);
    for (uint32_t k = 0; 64 * k < nsym; ++k) {
        const uint32_t CH = NX;
        NX = chunk(k + 1);
        const uint32_t i1 = min(64 * k + 64, nsym);
        for (uint32_t i = 64 * k; i < i1; ++i) {
            const uint32_t s = (srl(CH, (i >> 2) & 15u) >> (8u * (i & 3u))) & 0xffu;
            // CODEMPS / CODELPS (Annex C.2.4-C.2.5) + RENORME: with x = (MPS symbol) xor (A - Qe <
            // Qe), C takes Qe and A keeps A - Qe iff x, else A = Qe; the state moves unless the
            // symbol is an MPS that needs no renormalisation
            const uint32_t cx = s >> 1;
            const uint32_t e = srl(CTX, cx);
            const uint32_t qe = e & 0xffffu;
            const uint32_t a1 = q.a - qe;
            const bool ism = (s & 1u) == (e >> 31);
            const bool x = ism != (a1 < qe);
            const bool fast = ism && (a1 & 0x8000u);
            const uint32_t nidx = ism ? (e >> 16) & 0x7fu : (e >> 23) & 0x7fu;
            const uint32_t t0 = srl(TAB0, nidx & 63u), t1 = srl(TAB1, nidx & 63u);
            CTX = swl(CTX, fast ? e : ((nidx & 64u) ? t1 : t0), cx);
            const uint32_t an = x ? a1 : qe;
            q.c += x ? qe : 0u;
            uint32_t n = (uint32_t)__builtin_clz(an) - 16u;   // <= 15
            q.a = an << n;
            if (n >= q.ct) {   // a byte boundary: shift up to it, BYTEOUT (CT >= 7 after), maybe once more
                q.c <<= q.ct; n -= q.ct; q.byteout();
                if (n >= q.ct) { q.c <<= q.ct; n -= q.ct; q.byteout(); }
            }
            q.c <<= n; q.ct -= n;
            if (i + 1 == next_end)
                do close_pass(); while (p < npasses && next_end == i + 1);
        }
        lines_out((uint32_t)max(q.bp, 0) >> 6);
    }
    // the partial last line (bytes before bp are final; the stream ends at bp)
    const uint32_t nbytes = (uint32_t)q.bp;
    if (lf * 64 < nbytes && (uint32_t)(lane >> 4) == (lf & 3u) && lf * 64 + 4 * (lane & 15) + 4 <= cap &&
        (uint32_t)(lane & 15) * 4 < nbytes - lf * 64)
        *reinterpret_cast<uint32_t*>(out + (size_t)lf * 64 + 4 * (lane & 15)) = q.ring;
    __threadfence();
    if (lane != 0) return;
    uint32_t last = nbytes;
    for (int k = (int)npasses; k > 0;) {   // monotone rates (T1.cpp:907-919)
        GkPass& ps = P[--k];
        if (ps.rate > last) ps.rate = last; else last = ps.rate;
    }
    uint32_t prev = 0;
    for (uint32_t k = 0; k < npasses; ++k) {   // FF back-off (T1.cpp:920-930)
        GkPass& ps = P[k];
        if (ps.rate > 0 && ps.rate <= cap && out[ps.rate - 1] == 0xff) ps.rate--;
        ps.len = ps.rate - prev;
        prev = ps.rate;
    }
    info[4 * b] = numbps;
    info[4 * b + 1] = npasses;
    info[4 * b + 2] = P[npasses - 1].rate;
    info[4 * b + 3] = poff;
    if (nbytes > cap) atomicOr(err, 1);
}

// Outputs: info[4b..4b+3] = (numbps, npasses, bytes, offset of the block's
// passes in `passes`); pass records are packed (atomic offset allocation) so
// the host copies only the passes that exist.  With rate control the
// cumulative distortion follows T1::getwmsedec (T1.cpp:418-436, 836-842).
__global__ __launch_bounds__(256) void k_t1_mq(const uint8_t* __restrict__ sym, const uint64_t* __restrict__ sym_off,
                                              const uint32_t* __restrict__ pass_end, const uint32_t* __restrict__ cm_info,
                                              const GkBlock* __restrict__ blocks, uint8_t* __restrict__ bytes,
                                              GkPass* __restrict__ passes, uint32_t* __restrict__ info,
                                              uint32_t nblocks, int* err, const int32_t* __restrict__ pass_nmse,
                                              uint32_t* __restrict__ pass_counter, uint32_t nl,
                                              const uint32_t* __restrict__ order, uint32_t base, uint32_t count,
                                              uint32_t nsolo) {
    // nl = blocks per wave (lanes >= nl idle; gk_t1enc_lanes); pass ends staged in LDS [pass][lane].
    // A workgroup is four independent waves (one per SIMD) and takes a whole CU's LDS (the
    // launch pads it), so no other kernel's waves share a SIMD with an MQ chain.
    __shared__ MqLds Lw[4];
    extern __shared__ uint32_t pe_dyn[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the first nsolo waves (whole workgroups) are solo waves: position base + wave of `order`
    const uint32_t gw = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + wave));
    if (gw < nsolo) {
        if (gw < count)
            mq_solo_block(order ? order[base + gw] : base + gw, sym, sym_off, pass_end, cm_info, blocks, bytes, passes,
                          info, err, pass_nmse, pass_counter, lane);
        return;
    }
    MqLds& L = Lw[wave];
    for (int i = lane; i < MQ_PAIRS; i += 64) L.tab[i] = mq_pair_entry((uint32_t)i);
    // lane slot j = position base + nsolo + j of `order` (index order without one)
    base += nsolo;
    count = count > nsolo ? count - nsolo : 0;
    const uint32_t j = (gw - nsolo) * nl + lane;
    const bool inr = (uint32_t)lane < nl && j < count;
    const uint32_t b = inr ? (order ? order[base + j] : base + j) : 0xffffffffu;
    const bool has = inr && b < nblocks;
    uint32_t* pe_col = pe_dyn + (size_t)wave * (GK_MAX_PASSES + 1) * nl + (lane < (int)nl ? lane : 0);
#define pe_lds_at(p) pe_col[(size_t)(p) * nl]
    const uint32_t numbps = has ? cm_info[2 * b] : 0, npasses = has ? cm_info[2 * b + 1] : 0;
    const uint32_t* PE = pass_end + (size_t)(has ? b : 0) * GK_MAX_PASSES;
    for (uint32_t p = 0; p < npasses; ++p) pe_lds_at(p) = PE[p];
    if (has) pe_lds_at(npasses) = 0xffffffffu;
    const uint32_t nsym = npasses ? PE[npasses - 1] : 0;
    GkBlock B = {};
    if (has) B = blocks[b];
    const uint8_t* sp = sym + (has ? sym_off[b] : 0);
    uint32_t poff = 0;
    if (npasses) poff = atomicAdd(pass_counter, npasses);
    GkPass* P = passes + poff;
    const bool rc = (B.flags & 2) != 0;
    double cum = 0.0;
    MqLane q;
    // a lane without passes starts parked (no BYTEOUT ever; cap 0: no line leaves)
    q.a = 0x8000; q.c = 0; q.ct = npasses ? 12u : MQ_CT_PARKED; q.bp = -1; q.cur = 0; q.out = bytes + B.data_off;
    q.cap = has ? B.data_cap : 0;
    q.lf = 0;
    // initial context states (mqc_resetstates): every context at state 0 except ZC0 = 4, AGG = 3, UNI = 46
    for (int c = 0; c < 19; ++c)
        L.ctx[c][lane] = mq_pair_entry(2 * (c == CTX_ZC ? 4 : (c == CTX_AGG ? 3 : (c == CTX_UNI ? 46 : 0))));
    uint32_t maxsym = nsym;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxsym = max(maxsym, (uint32_t)__shfl_xor((int)maxsym, o));
    __syncthreads();
    uint32_t p = 0, next_end = has ? pe_lds_at(0) : 0xffffffffu;
    // pass bookkeeping (T1.cpp:856-897); only the last pass is terminated (default style)
    auto close_passes = [&](uint32_t i) {
        while (__any(npasses && p < npasses && next_end == i)) {
            if (npasses && p < npasses && next_end == i) {
                if (p == npasses - 1) {   // FLUSH (Annex C.2.9, mqc_enc.cpp:229-247), C as 32 bits
                    uint32_t tempc = q.c + q.a;
                    uint32_t c32 = q.c | 0xffff;
                    if (c32 >= tempc) c32 -= 0x8000;
                    uint32_t c = c32 << q.ct, ct = 0;
                    mq_byteout5(q, L, lane, ~0u, c, ct);
                    c <<= ct; ct = 0;
                    mq_byteout5(q, L, lane, ~0u, c, ct);
                    q.c = c; q.ct = ct;
                    if (q.cur != 0xff) { mq_put5(q, L, lane, ~0u, q.cur); q.cur = 0; }
                    P[p].rate = (uint32_t)q.bp;
                    q.ct = MQ_CT_PARKED;   // the block is coded: no BYTEOUT from here on
                } else {
                    P[p].rate = (uint32_t)q.bp + 5 + (q.ct < 5 ? 1 : 0);
                }
                if (rc) {
                    const int bpno = p == 0 ? (int)numbps - 1 : (int)numbps - 2 - (int)(p - 1) / 3;
                    // Grok's roundings, one per operation (no fused multiply-add): the values feed
                    // PCRD on the host and the plugin tree's distortionDecrease
                    double wm = __dmul_rn(B.wmse, (double)(1 << bpno));
                    wm = __dmul_rn(wm, __dmul_rn(wm, (double)pass_nmse[(size_t)b * GK_MAX_PASSES + p]) / 8192.0);
                    cum = __dadd_rn(cum, wm);
                }
                P[p].dist = cum;
                ++p;
                next_end = pe_lds_at(p);
            }
        }
    };
    close_passes(0);   // passes without symbols before the first one
    // earliest pass end of the wave (uniform), so the per-symbol test is one scalar compare
    auto wave_next_end = [&]() -> uint32_t {
        uint32_t m = (npasses && p < npasses) ? next_end : 0xffffffffu;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o));
        return __builtin_amdgcn_readfirstlane(m);
    };
    uint32_t wnext = wave_next_end();
    uint4 cur4 = make_uint4(0, 0, 0, 0), nxt4 = make_uint4(0, 0, 0, 0);
    if (nsym) cur4 = *(const uint4*)(sp);
    if (nsym > 16) nxt4 = *(const uint4*)(sp + 16);
    q.pcx1 = 19; q.pne1 = 0;
    q.epref = L.ctx[min(byte_of(cur4, 0) >> 1, 19u)][lane];
    for (uint32_t base = 0; base < maxsym; base += 16) {
        uint4 pre = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) {
            const uint32_t i = base + j;
            mq_code5(q, L, lane, byte_of(cur4, j), byte_of(j < 15 ? cur4 : nxt4, (j + 1) & 15));
            // the prefetch two chunks ahead is issued after the first symbol has consumed this
            // chunk's bytes, so the wait for them does not also wait for the prefetch
            if (j == 0) {
                __builtin_amdgcn_sched_barrier(0);
                if (base + 32 < nsym) pre = *(const uint4*)(sp + base + 32);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (i + 1 == wnext) { close_passes(i + 1); wnext = wave_next_end(); }
        }
        cur4 = nxt4; nxt4 = pre;
        mq_lines_out(q, L, lane);
    }
    // the partial last line: whole dwords before bp, then the dword holding bp (pending byte)
    if (npasses && q.bp >= 0 && (uint32_t)q.bp < q.cap) {
        const uint32_t bp = (uint32_t)q.bp, cl = bp >> 6;
        reinterpret_cast<uint8_t*>(&L.ring[lane][0])[bp & (4 * MQ_RING_DW - 1)] = (uint8_t)q.cur;
        if (cl > q.lf) mq_line_store(q, L, lane, q.lf);
        const uint32_t o = (cl & 1) * 16, k = (bp >> 2) & 15;
        for (uint32_t i = 0; i <= k; ++i) *(uint32_t*)(q.out + (size_t)cl * 64 + 4 * i) = L.ring[lane][o + i];
    }
    if (!has) return;
    if (npasses == 0) { info[4 * b] = 0; info[4 * b + 1] = 0; info[4 * b + 2] = 0; info[4 * b + 3] = 0; return; }
    __threadfence();
    const uint32_t nbytes = (uint32_t)q.bp;
    uint32_t last = nbytes;
    for (int k = (int)npasses; k > 0;) {   // monotone rates (T1.cpp:907-919)
        GkPass& ps = P[--k];
        if (ps.rate > last) ps.rate = last; else last = ps.rate;
    }
    uint32_t prev = 0;
    for (uint32_t k = 0; k < npasses; ++k) {   // FF back-off (T1.cpp:920-930)
        GkPass& ps = P[k];
        if (ps.rate > 0 && ps.rate <= q.cap && q.out[ps.rate - 1] == 0xff) ps.rate--;
        ps.len = ps.rate - prev;
        prev = ps.rate;
    }
    info[4 * b] = numbps;
    info[4 * b + 1] = npasses;
    info[4 * b + 2] = P[npasses - 1].rate;
    info[4 * b + 3] = poff;
    if (q.bp > 0 && (uint32_t)q.bp > q.cap) atomicOr(err, 1);
#undef pe_lds_at
}

#include "gk_launch.h"
void gk_launch_t1_cm(hipStream_t st, const int32_t* coef, const GkBlock* blocks, const uint64_t* sym_off, uint8_t* sym,
                     uint32_t* pass_end, uint32_t* cm_info, uint32_t nblocks, int* err, const int16_t* nmse_tab,
                     int32_t* pass_nmse, const uint32_t* order, uint32_t base, uint32_t count) {
    if (!nblocks) return;
    if (count == 0xffffffffu) count = nblocks;
    if (!count) return;
    if (pass_nmse)
        hipLaunchKernelGGL(k_t1_cm<true>, dim3(count), dim3(64), 0, st, coef, blocks, sym_off, sym, pass_end, cm_info,
                           nblocks, err, nmse_tab, pass_nmse, order, base, count);
    else
        hipLaunchKernelGGL(k_t1_cm<false>, dim3(count), dim3(64), 0, st, coef, blocks, sym_off, sym, pass_end,
                           cm_info, nblocks, err, nmse_tab, pass_nmse, order, base, count);
}

// Per block an estimate of the MQ decisions T1 will code, as the weight that orders the chunked
// context-modelling / MQ overlap (one wave per block).  With P coded bit-planes every sample
// takes about one decision per plane - zero coding above its most significant bit, then the
// significance, its sign and the refinements - except the zeros a run-length column codes four
// at a time; samples with more magnitude bits leave fewer such zeros.  Weight, in eighths of a
// decision: 5 P area + 3 (sum of the samples' magnitude bit counts), i.e. P decisions per sample
// less 3/8 of the zeros above the samples' most significant bits.  The estimate only orders the
// blocks (each is coded the same whatever the order), so it is taken over every fourth row - a
// quarter of the coefficient lines - with the bit count scaled back (a full pass was 0.28 ms of
// C2's encode, `profiles/r04z_C2_kernel_stats.txt`).
__global__ __launch_bounds__(64) void k_t1_weight(const int32_t* __restrict__ coef, const GkBlock* __restrict__ blocks,
                                                  uint32_t* __restrict__ weight, uint32_t nblocks) {
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const int lane = threadIdx.x;
    const GkBlock B = blocks[b];
    const bool irrev = B.flags & 1;
    uint32_t mx = 0, nbits = 0;
    if (lane < (int)B.w)
#pragma unroll 4
        for (uint32_t y = 0; y < B.h; y += 4) {
            const int32_t raw = coef[B.band_off + (size_t)y * B.stride + lane];
            const uint32_t a0 = irrev ? (uint32_t)fabsf(rintf((__int_as_float(raw) / B.step) * 64.0f))
                                      : (uint32_t)(raw < 0 ? -raw : raw) * 64u;
            const uint32_t a = ((a0 >> 6) << (6 + (B.flags >> 3))) | (a0 & 63u);   // ROI maxshift
            mx = a > mx ? a : mx;
            nbits += (a >> 6) ? 32u - __clz(a >> 6) : 0u;
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t t = __shfl_xor(mx, o); mx = t > mx ? t : mx;
        nbits += __shfl_xor(nbits, o);
    }
    if (lane == 0) {
        const uint32_t t = mx ? 32 - __clz(mx) : 0;
        const uint32_t planes = t <= 6 ? 0 : t - 6;
        const uint32_t rows = (B.h + 3) / 4;   // rows sampled
        weight[b] = planes * B.w * B.h * 5u + (uint32_t)((3ull * nbits * B.h) / (rows ? rows : 1));
    }
}
void gk_launch_t1_weight(hipStream_t st, const int32_t* coef, const GkBlock* blocks, uint32_t* weight, uint32_t nblocks) {
    if (!nblocks) return;
    hipLaunchKernelGGL(k_t1_weight, dim3(nblocks), dim3(64), 0, st, coef, blocks, weight, nblocks);
}
void gk_launch_t1_mq(hipStream_t st, const uint8_t* sym, const uint64_t* sym_off, const uint32_t* pass_end,
                     const uint32_t* cm_info, const GkBlock* blocks, uint8_t* bytes, GkPass* passes, uint32_t* info,
                     uint32_t nblocks, int* err, const int32_t* pass_nmse, uint32_t* pass_counter, const uint32_t* order,
                     uint32_t base, uint32_t count, uint32_t nsolo) {
    if (!nblocks) return;
    if (count == 0xffffffffu) count = nblocks;
    if (!count) return;
    nsolo = std::min((nsolo + 3) / 4 * 4, (count + 3) / 4 * 4);   // whole workgroups of solo waves
    static uint32_t nl = 0;
    if (!nl) {   // blocks per 64-lane wave (GK_T1ENC_LANES, 1..64)
        const char* v = getenv("GK_T1ENC_LANES");
        const int n = v ? atoi(v) : 64;
        nl = (uint32_t)(n < 1 ? 1 : (n > 64 ? 64 : n));
    }
    // dynamic LDS: the four waves' pass ends, padded so one workgroup fills the CU's 160 KiB
    const size_t pe = (size_t)(GK_MAX_PASSES + 1) * nl * 4 * 4;
    const size_t lds = std::max(pe, (size_t)163840 - 4 * sizeof(MqLds));
    const uint32_t rest = count > nsolo ? count - nsolo : 0;
    hipLaunchKernelGGL(k_t1_mq, dim3(nsolo / 4 + (rest + 4 * nl - 1) / (4 * nl)), dim3(256), lds, st, sym, sym_off,
                       pass_end, cm_info, blocks, bytes, passes, info, nblocks, err, pass_nmse, pass_counter, nl, order,
                       base, count, nsolo);
}
