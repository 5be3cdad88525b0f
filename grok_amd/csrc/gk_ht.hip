// gk_ht.hip — HTJ2K block coder (ISO/IEC 15444-15 cleanup pass) for gfx950.
//
// Grok 9.2.0 codes HT blocks with OpenJPH 0.7.2 (t1/t1_ht/T1HT.cpp:109-187 ->
// ojph_encode_codeblock / ojph_decode_codeblock): one cleanup pass per block,
// three byte streams — MagSgn (forward, bit-stuffed after 0xFF), MEL (adaptive
// run-length, forward) and VLC (CxtVLC + U-VLC, written backward) — laid out as
// MagSgn | MEL | VLC with the 12-bit interface locator Scup in the last two bytes.
//
// Mapping: one lane per code-block (64 blocks per wave).  Every lane walks its
// block's quad pairs in the same order, so the quad loop is uniform across the
// wave; the per-lane line state (exponent and context bytes of the previous
// quad row) lives in LDS as [entry][lane] columns (conflict-free), and the
// CxtVLC lookup tables are copied into LDS once per workgroup.
//
// Encoder outputs per block (slot = [data_off, data_off + data_cap)):
//   MagSgn bytes at the slot start, the MEL+VLC tail (Scup bytes) at the slot
//   end; info = {numbps 1, npasses 1, total bytes, MagSgn bytes}.  The host T2
//   emits the two pieces back to back, which is the block's codeword segment.
// Decoder: reads one contiguous block segment (gathered by T2) and writes the
//   signed coefficients straight into the band window of the arena.
#include <hip/hip_runtime.h>
#include "gk_common.h"
#include "gk_launch.h"
#define GK_HT_TABLE_QUAL __constant__
#include "gk_ht_tables.h"

// Workgroup size and line-state entries per lane (w/2 + 4): 256 lanes x 36 entries for blocks up
// to 64 wide; code-blocks up to 1024 wide (Grok accepts 4 <= w, h <= 1024 with w * h <= 4096,
// grk_compress.cpp:981-988) take 64-lane workgroups with 516 entries (66 KB of line state)
#define HT_WG_STD 256
#define HT_LINE_STD 36
#define HT_WG_WIDE 64
#define HT_LINE_WIDE 516
#ifndef HT_OUTC
#define HT_OUTC 16          // decoder output staging: columns per flush (8 or 16)
#endif

// MEL exponent table {0,0,0,1,1,1,2,2,2,3,3,4,5} packed 3 bits per state
__device__ __forceinline__ int mel_exp(int k) {
    const uint64_t T = (0ull) | (0ull << 3) | (0ull << 6) | (1ull << 9) | (1ull << 12) | (1ull << 15) | (2ull << 18) |
                       (2ull << 21) | (2ull << 24) | (3ull << 27) | (3ull << 30) | (4ull << 33) | (5ull << 36);
    return (int)((T >> (3 * k)) & 7);
}

// U-VLC code of u (clause 7.3.6): prefix "1", "01", "001"+1 bit, "000"+5 bits,
// bits emitted LSB first.  Returns the prefix in (pre, plen), suffix in (suf, slen).
__device__ __forceinline__ void uvlc_code(int u, uint32_t& pre, int& plen, uint32_t& suf, int& slen) {
    if (u <= 0) { pre = 0; plen = 0; suf = 0; slen = 0; }
    else if (u == 1) { pre = 1; plen = 1; suf = 0; slen = 0; }
    else if (u == 2) { pre = 2; plen = 2; suf = 0; slen = 0; }
    else if (u <= 4) { pre = 4; plen = 3; suf = (uint32_t)(u - 3); slen = 1; }
    else { pre = 0; plen = 3; suf = (uint32_t)(u - 5); slen = 5; }
}

// =============================================================================
// Encoder
// =============================================================================
template <int HT_WG, int HT_LINE>
__global__ __launch_bounds__(HT_WG) void k_ht_enc(const int32_t* __restrict__ coef, const GkBlock* __restrict__ blocks,
                                                  uint8_t* __restrict__ bytes, uint8_t* __restrict__ mel_scratch,
                                                  uint32_t mel_cap, uint32_t* __restrict__ info, uint32_t nblocks,
                                                  int* __restrict__ err, uint32_t nl) {
    __shared__ uint16_t s_tab[2][2048];
    __shared__ uint8_t s_e[HT_LINE][HT_WG];
    __shared__ uint8_t s_cx[HT_LINE][HT_WG];
    // Input staging: a lane's 8 columns x 2 rows, loaded as two 16-byte pieces per row when its
    // quads reach them (a 4-byte load per sample was a 64-line gather, one block per lane).
    __shared__ int32_t s_in[2][8][HT_WG];
    // Output staging: the lane's current 64-byte block of the MagSgn and of the VLC stream
    // (four 16-byte lines each), stored to HBM as four consecutive 16-byte stores once complete
    __shared__ uint4 s_ms[4][HT_WG], s_v[4][HT_WG];
    const int tid = threadIdx.x;
    for (int i = tid; i < 2048; i += HT_WG) { s_tab[0][i] = HT_VLC_ENC0[i]; s_tab[1][i] = HT_VLC_ENC1[i]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) s_v[i][tid] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    // nl blocks per wave (the other lanes idle): more, thinner waves per SIMD hide the serial
    // coder's memory waits behind each other (GK_HT_LANES)
    const uint32_t b = (blockIdx.x * (HT_WG / 64) + (tid >> 6)) * nl + (tid & 63);
    if ((uint32_t)(tid & 63) >= nl || b >= nblocks) return;

    const GkBlock G = blocks[b];
    const int32_t* src = coef + G.band_off;
    const uint32_t stride = G.stride, w = G.w, h = G.h;
    uint8_t* slot = bytes + G.data_off;
    uint8_t* tail_end = slot + G.data_cap;
    uint8_t* mel = mel_scratch + (size_t)b * mel_cap;
    bool ovf = false;

    // Output bytes leave in whole 64-byte blocks: each stream collects its bytes in a 16-byte
    // register line aligned like its destination, a complete line goes to the lane's LDS block,
    // and a complete block leaves as four consecutive 16-byte stores.  (One block per lane
    // makes every store instruction a 64-line scatter; byte stores, and then single 16-byte
    // lines, left partial lines in L2 that were written back more than once: the encoder wrote
    // 3.4x its output, `profiles/r04s_C4_pmc.txt`, `r05_C4_pmc.txt`.)
    // ---- MagSgn: LSB-first, a byte after 0xFF carries 7 bits; forward from the slot start
    // (64-byte aligned)
    uint64_t ms_acc = 0; int ms_n = 0, ms_k = 8; uint32_t ms_pos = 0;
    uint64_t ms_l0 = 0, ms_l1 = 0;   // the current line, bytes ms_pos & ~15 ..
    auto ms_byte = [&](uint32_t byte) {
        const uint32_t o = ms_pos & 15;
        if (o < 8) ms_l0 |= (uint64_t)byte << (8 * o); else ms_l1 |= (uint64_t)byte << (8 * (o - 8));
        ++ms_pos;
        if ((ms_pos & 15) == 0) {
            s_ms[((ms_pos - 16) >> 4) & 3][tid] = make_uint4((uint32_t)ms_l0, (uint32_t)(ms_l0 >> 32), (uint32_t)ms_l1, (uint32_t)(ms_l1 >> 32));
            ms_l0 = ms_l1 = 0;
            if ((ms_pos & 63) == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i) *(uint4*)(slot + ms_pos - 64 + 16 * i) = s_ms[i][tid];
            }
        }
    };
    auto ms_put = [&](uint32_t v, int m) {
        ms_acc |= (uint64_t)v << ms_n; ms_n += m;
        while (ms_n >= ms_k) {
            uint32_t byte = (uint32_t)ms_acc & ((1u << ms_k) - 1);
            ms_acc >>= ms_k; ms_n -= ms_k;
            ms_byte(byte);
            ms_k = (byte == 0xFF) ? 7 : 8;
        }
    };
    // ---- VLC: LSB-first, grows backward from the slot end; after a byte > 0x8F the
    // next byte's MSB is a stuffed 0 unless its low 7 bits differ from 0x7F.  Byte i goes to
    // tail_end - 2 - i; the register line holds the 16-byte aligned line of the current byte, a
    // line the stream moves below goes to the LDS block, and the block leaves once its lowest
    // line is complete.  (Lines of a block above the slot end lie in the padding before the
    // next 64-byte aligned slot; the locator bytes are stored last.)
    uint64_t v_acc = 0xF; int v_n = 4; bool v_gt = true; uint32_t v_cnt = 0, v_first = 0;
    uint64_t v_l0 = 0, v_l1 = 0;
    uint8_t* v_line = (uint8_t*)((uintptr_t)(tail_end - 2) & ~(uintptr_t)15);
    auto v_emit = [&](uint32_t byte) {
        if (v_cnt == 0) v_first = byte;
        uint8_t* a = tail_end - 2 - (int)v_cnt;
        if (a < v_line) {   // the line above is complete
            s_v[((uintptr_t)v_line >> 4) & 3][tid] = make_uint4((uint32_t)v_l0, (uint32_t)(v_l0 >> 32), (uint32_t)v_l1, (uint32_t)(v_l1 >> 32));
            if (((uintptr_t)v_line & 63) == 0) {   // its block is complete
#pragma unroll
                for (int i = 0; i < 4; ++i) *(uint4*)(v_line + 16 * i) = s_v[i][tid];
            }
            v_l0 = v_l1 = 0;
            v_line -= 16;
        }
        const uint32_t o = (uint32_t)(a - v_line);
        if (o < 8) v_l0 |= (uint64_t)byte << (8 * o); else v_l1 |= (uint64_t)byte << (8 * (o - 8));
        ++v_cnt;
    };
    auto vlc_put = [&](uint32_t cw, int len) {
        v_acc |= (uint64_t)cw << v_n; v_n += len;
        while (v_n >= 8) {
            uint32_t byte; int used;
            if (v_gt && (v_acc & 0x7F) == 0x7F) { byte = 0x7F; used = 7; }
            else { byte = (uint32_t)v_acc & 0xFF; used = 8; }
            v_acc >>= used; v_n -= used;
            v_emit(byte);
            v_gt = byte > 0x8F;
        }
    };
    // ---- MEL: MSB-first bits, a byte after 0xFF carries 7 bits
    // (staged in the block's scratch a dword at a time; copied into place once Scup is known)
    uint32_t m_tmp = 0, m_cnt = 0, m_word = 0; int m_rem = 8, m_run = 0, m_k = 0, m_thr = 1;
    auto mel_store = [&](uint32_t byte) {
        m_word |= byte << (8 * (m_cnt & 3));
        ++m_cnt;
        if ((m_cnt & 3) == 0) {
            if (m_cnt <= mel_cap) *(uint32_t*)(mel + m_cnt - 4) = m_word; else ovf = true;
            m_word = 0;
        }
    };
    auto mel_bit = [&](int v) {
        m_tmp = (m_tmp << 1) | (uint32_t)v;
        if (--m_rem == 0) { mel_store(m_tmp); m_rem = (m_tmp == 0xFF) ? 7 : 8; m_tmp = 0; }
    };
    auto mel_code = [&](bool one) {
        if (!one) {
            if (++m_run >= m_thr) { mel_bit(1); m_run = 0; m_k = min(12, m_k + 1); m_thr = 1 << mel_exp(m_k); }
        } else {
            mel_bit(0);
            for (int t = mel_exp(m_k); t > 0;) mel_bit((m_run >> --t) & 1);
            m_run = 0; m_k = max(0, m_k - 1); m_thr = 1 << mel_exp(m_k);
        }
    };

    // 9/7: the quantisation index of T1HT::preCompress (T1HT.cpp:88-104) taken from the float
    // coefficient, trunc(x * (1 / stepsize)) (R-BUG-2: Grok reads the float bits as an int)
    const bool irrev = G.flags & 1;
    const float inv_step = irrev ? 1.0f / G.step : 0.0f;
    // ROI maxshift (the component is the region): every index magnitude scaled up by 2^shift, the
    // band's bit-plane count raised by it (standard-correct; Grok's encoder only raises the count)
    const uint32_t rshift = G.flags >> 3;
    // columns [x8, x8 + 8) of rows y, y + 1 into the staging (zeros outside the block)
    auto stage = [&](uint32_t x8, uint32_t y) {
        const uint32_t nc = x8 < w ? min(8u, w - x8) : 0u;
        for (uint32_t r = 0; r < 2; ++r) {
            const int32_t* row = src + (size_t)(y + r) * stride + x8;
            if (y + r < h && nc == 8 && ((uintptr_t)row & 15) == 0) {
                const uint4 a = reinterpret_cast<const uint4*>(row)[0], c = reinterpret_cast<const uint4*>(row)[1];
                s_in[r][0][tid] = (int32_t)a.x; s_in[r][1][tid] = (int32_t)a.y; s_in[r][2][tid] = (int32_t)a.z;
                s_in[r][3][tid] = (int32_t)a.w; s_in[r][4][tid] = (int32_t)c.x; s_in[r][5][tid] = (int32_t)c.y;
                s_in[r][6][tid] = (int32_t)c.z; s_in[r][7][tid] = (int32_t)c.w;
            } else {
                for (uint32_t k = 0; k < 8; ++k) s_in[r][k][tid] = (y + r < h && k < nc) ? row[k] : 0;
            }
        }
    };
    auto ld = [&](uint32_t x, uint32_t y) -> int32_t {
        const int32_t raw = s_in[y & 1][x & 7][tid];
        const int32_t v = irrev ? (int32_t)(__int_as_float(raw) * inv_step) : raw;
        return v < 0 ? -(int32_t)((uint32_t)-v << rshift) : (int32_t)((uint32_t)v << rshift);
    };
    // one quad: samples (x,y) (x,y+1) (x+1,y) (x+1,y+1) -> rho, exponents, MagSgn values
    auto quad = [&](uint32_t x, uint32_t y, int& rho, int* e, uint32_t* sv, int& emax) {
        int32_t v[4] = {ld(x, y), ld(x, y + 1), ld(x + 1, y), ld(x + 1, y + 1)};
        rho = 0; emax = 0;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            uint32_t mu = (uint32_t)(v[n] < 0 ? -v[n] : v[n]);
            int en = mu ? 32 - __clz(2 * mu - 1) : 0;
            rho |= (mu ? 1 : 0) << n;
            e[n] = en;
            emax = max(emax, en);
            sv[n] = mu ? 2 * mu - 2 + (v[n] < 0 ? 1u : 0u) : 0u;
        }
    };
    auto ms_quad = [&](int rho, int Uq, uint32_t tup, const uint32_t* sv) {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            int m = ((rho >> n) & 1) ? Uq - (int)((tup >> n) & 1) : 0;
            if (m) ms_put((uint32_t)(sv[n] & (uint32_t)((1ull << m) - 1)), m);
        }
    };

    int c_q0 = 0;
    for (uint32_t y = 0; y < h; y += 2) {
        const bool first = y == 0;
        const uint16_t* tbl = s_tab[first ? 0 : 1];
        int max_e = 0;
        if (!first) {
            max_e = max((int)s_e[0][tid], (int)s_e[1][tid]) - 1;
            s_e[0][tid] = 0;
            c_q0 = s_cx[0][tid] + (s_cx[1][tid] << 2);
            s_cx[0][tid] = 0;
        } else {
            s_e[0][tid] = 0; s_cx[0][tid] = 0;
        }
        uint32_t li = 0;
        for (uint32_t x = 0; x < w; x += 4) {
            int rho0, rho1 = 0, e[8], emax0, emax1 = 0;
            uint32_t sv[8];
            if ((x & 7) == 0) stage(x, y);
            quad(x, y, rho0, e, sv, emax0);
            const int kappa0 = (first || !(rho0 & (rho0 - 1))) ? 1 : max(1, max_e);
            const int Uq0 = max(emax0, kappa0), u0 = Uq0 - kappa0;
            int eps0 = 0;
            if (u0 > 0) {
#pragma unroll
                for (int n = 0; n < 4; ++n) eps0 |= (e[n] == emax0) << n;
            }
            s_e[li][tid] = (uint8_t)max((int)s_e[li][tid], e[1]);
            ++li;
            if (!first) max_e = max((int)s_e[li][tid], (int)s_e[li + 1][tid]) - 1;
            s_e[li][tid] = (uint8_t)e[3];
            s_cx[li - 1][tid] = (uint8_t)(s_cx[li - 1][tid] | ((rho0 & 2) >> 1));
            int c_q1 = first ? 0 : s_cx[li][tid] + (s_cx[li + 1][tid] << 2);
            s_cx[li][tid] = (uint8_t)((rho0 & 8) >> 3);
            const uint32_t t0 = tbl[(c_q0 << 8) + (rho0 << 4) + eps0];
            uint32_t cw = t0 >> 8; int clen = (t0 >> 4) & 7;
            if (c_q0 == 0) mel_code(rho0 != 0);
            ms_quad(rho0, Uq0, t0, sv);
            int u1 = 0;
            if (x + 2 < w) {
                quad(x + 2, y, rho1, e + 4, sv + 4, emax1);
                const int kappa1 = (first || !(rho1 & (rho1 - 1))) ? 1 : max(1, max_e);
                if (first) c_q1 = (rho0 >> 1) | (rho0 & 1);
                else c_q1 |= ((rho0 & 4) >> 1) | ((rho0 & 8) >> 2);
                const int Uq1 = max(emax1, kappa1);
                u1 = Uq1 - kappa1;
                int eps1 = 0;
                if (u1 > 0) {
#pragma unroll
                    for (int n = 0; n < 4; ++n) eps1 |= (e[4 + n] == emax1) << n;
                }
                s_e[li][tid] = (uint8_t)max((int)s_e[li][tid], e[5]);
                ++li;
                if (!first) max_e = max((int)s_e[li][tid], (int)s_e[li + 1][tid]) - 1;
                s_e[li][tid] = (uint8_t)e[7];
                s_cx[li - 1][tid] = (uint8_t)(s_cx[li - 1][tid] | ((rho1 & 2) >> 1));
                if (!first) c_q0 = s_cx[li][tid] + (s_cx[li + 1][tid] << 2);
                s_cx[li][tid] = (uint8_t)((rho1 & 8) >> 3);
                const uint32_t t1 = tbl[(c_q1 << 8) + (rho1 << 4) + eps1];
                cw |= (t1 >> 8) << clen; clen += (t1 >> 4) & 7;
                if (c_q1 == 0) mel_code(rho1 != 0);
                ms_quad(rho1, Uq1, t1, sv + 4);
            }
            // both CxtVLC codewords, then the U-VLC codes of the pair, in one VLC append
            uint32_t p0, s0, p1, s1; int pl0, sl0, pl1, sl1;
            if (first && u0 > 0 && u1 > 0) {
                mel_code(min(u0, u1) > 2);
                if (u0 > 2 && u1 > 2) {
                    uvlc_code(u0 - 2, p0, pl0, s0, sl0); uvlc_code(u1 - 2, p1, pl1, s1, sl1);
                } else if (u0 > 2) {
                    uvlc_code(u0, p0, pl0, s0, sl0);
                    p1 = (uint32_t)(u1 - 1); pl1 = 1; s1 = 0; sl1 = 0;
                } else {
                    uvlc_code(u0, p0, pl0, s0, sl0); uvlc_code(u1, p1, pl1, s1, sl1);
                }
            } else {
                uvlc_code(u0, p0, pl0, s0, sl0); uvlc_code(u1, p1, pl1, s1, sl1);
            }
            uint64_t all = (uint64_t)cw | ((uint64_t)p0 << clen);
            int n = clen + pl0;
            all |= (uint64_t)p1 << n; n += pl1;
            all |= (uint64_t)s0 << n; n += sl0;
            all |= (uint64_t)s1 << n; n += sl1;
            vlc_put((uint32_t)all, n);   // n <= 7 + 7 + 3 + 3 + 5 + 5 = 30
            if (first) c_q0 = (rho1 >> 1) | (rho1 & 1);
            else c_q0 |= ((rho1 & 4) >> 1) | ((rho1 & 8) >> 2);
        }
        if (first) s_e[li + 1][tid] = 0;
    }

    // ---- termination (MEL + VLC fuse, MagSgn padding)
    if (m_run > 0) mel_bit(1);
    if (v_gt && v_n == 7 && (v_acc & 0x7F) == 0x7F) { v_emit(0x7F); v_acc = 0; v_n = 0; v_gt = false; }
    {
        const uint32_t mtmp = (m_tmp << m_rem) & 0xFF, vtmp = (uint32_t)v_acc & 0xFF;
        const uint32_t mel_mask = (0xFFu << m_rem) & 0xFF, vlc_mask = 0xFFu >> (8 - v_n);
        if (mel_mask | vlc_mask) {
            const uint32_t fuse = mtmp | vtmp;
            if (((((fuse ^ mtmp) & mel_mask) | ((fuse ^ vtmp) & vlc_mask)) == 0) && fuse != 0xFF && v_cnt > 0) {
                mel_store(fuse);
            } else {
                mel_store(mtmp);
                v_emit(vtmp);
            }
        }
    }
    if (ms_n > 0) {
        const int t = ms_k - ms_n;
        const uint32_t byte = ((uint32_t)ms_acc | (((1u << t) - 1) << ms_n)) & 0xFF;
        if (byte != 0xFF) ms_byte(byte);
    }
    // the MagSgn block in progress: its complete lines from LDS, then the line in progress up to
    // ms_pos, dword by dword (a block just completed has been stored)
    for (uint32_t i = 0; i < ((ms_pos & 63) >> 4); ++i) *(uint4*)(slot + (ms_pos & ~63u) + 16 * i) = s_ms[i][tid];
    for (uint32_t d = 0; d < ((ms_pos & 15) + 3) / 4; ++d)
        *(uint32_t*)(slot + (ms_pos & ~15u) + 4 * d) = (uint32_t)((d < 2 ? ms_l0 : ms_l1) >> (32 * (d & 1)));
    if (ms_n == 0 && ms_k == 7) --ms_pos;   // a trailing 0xFF is dropped (it stays stored, past ms_pos)
    if (m_cnt & 3) {   // the MEL dword in progress
        if (m_cnt <= mel_cap) *(uint32_t*)(mel + (m_cnt & ~3u)) = m_word; else ovf = true;
    }
    const uint32_t scup = m_cnt + v_cnt + 1;
    if (ovf || (uint64_t)ms_pos + scup > G.data_cap || scup > 4079) {
        atomicOr(err, 1);
        info[4 * (size_t)b + 0] = 1; info[4 * (size_t)b + 1] = 0; info[4 * (size_t)b + 2] = 0; info[4 * (size_t)b + 3] = 0;
        return;
    }
    // the VLC block in progress: its complete lines above the current one from LDS (lines above
    // the stream's first are zero: padding or the locator bytes stored below), then the line in
    // progress: its bytes from the last one up to the line's top (or the slot end), one by one -
    // MEL bytes go right below them
    for (uint8_t* L = v_line + 16; ((uintptr_t)L & 63) != 0; L += 16) *(uint4*)L = s_v[((uintptr_t)L >> 4) & 3][tid];
    {
        uint8_t* lo = tail_end - 1 - (int)v_cnt;   // the last VLC byte
        uint8_t* hi = v_line + 16 < tail_end ? v_line + 16 : tail_end;
        for (uint8_t* a = lo; a < hi; ++a) {
            const uint32_t o = (uint32_t)(a - v_line);
            *a = (uint8_t)((o < 8 ? v_l0 >> (8 * o) : v_l1 >> (8 * (o - 8))) & 0xFF);
        }
    }
    uint8_t* tail = tail_end - scup;
    for (uint32_t i = 0; i < m_cnt; ++i) tail[i] = mel[i];
    tail_end[-1] = (uint8_t)(scup >> 4);
    tail_end[-2] = (uint8_t)((v_first & 0xF0) | (scup & 0xF));
    info[4 * (size_t)b + 0] = 1;                    // cblk->numbps = 1 (T1HT.cpp:128)
    info[4 * (size_t)b + 1] = 1;                    // one cleanup pass
    info[4 * (size_t)b + 2] = ms_pos + scup;        // Lcup
    info[4 * (size_t)b + 3] = ms_pos;               // MagSgn bytes (head piece)
}

// =============================================================================
// Decoder
// =============================================================================
template <int HT_WG, int HT_LINE>
__global__ __launch_bounds__(HT_WG) void k_ht_dec(const uint8_t* __restrict__ bytes, const GkBlock* __restrict__ blocks,
                                                  const uint32_t* __restrict__ ids, int32_t* __restrict__ coef,
                                                  uint32_t nblocks, int* __restrict__ err, uint32_t nl) {
    __shared__ uint16_t s_tab[2][1024];
    __shared__ uint8_t s_e[HT_LINE][HT_WG];
    __shared__ uint8_t s_cx[HT_LINE][HT_WG];
    // Output staging: a lane's samples of HT_OUTC columns x 2 rows, stored as HT_OUTC / 4 16-byte
    // pieces per row once those columns are decoded.  Storing each sample as it is decoded made
    // every store a 64-line scatter (one block per lane): C4 k_ht_dec 9.0 ms, 4.9 ms with no stores
    // at all; 8 columns (32 bytes per row and flush) wrote 1.5x the samples (partial 128-byte lines
    // written back more than once, `profiles/r05b_C4_pmc.txt`), 16 columns write half lines.
    __shared__ uint32_t s_out[2][HT_OUTC][HT_WG];
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024; i += HT_WG) { s_tab[0][i] = HT_VLC_DEC0[i]; s_tab[1][i] = HT_VLC_DEC1[i]; }
    __syncthreads();
    // nl blocks per wave (the other lanes idle): more, thinner waves per SIMD hide the serial
    // coder's memory waits behind each other (GK_HT_LANES)
    const uint32_t b = (blockIdx.x * (HT_WG / 64) + (tid >> 6)) * nl + (tid & 63);
    if ((uint32_t)(tid & 63) >= nl || b >= nblocks) return;

    const GkBlock G = blocks[ids ? ids[b] : b];
    int32_t* dst = coef + G.band_off;
    const uint32_t stride = G.stride, w = G.w, h = G.h;
    auto zero_block = [&]() {
        for (uint32_t y = 0; y < h; ++y)
            for (uint32_t x = 0; x < w; ++x) dst[(size_t)y * stride + x] = 0;
    };
    const uint32_t lcup = G.len;
    // Grok hands every byte to the cleanup pass (T1HT::decompress, T1HT.cpp:169-173: lengths1 =
    // all bytes, lengths2 = 0), so a block with SigProp / MagRef passes is an error
    // (ojph_block_decoder.cpp:1014-1019), as here
    if (G.npasses > 1 && lcup) { atomicOr(err, 4); zero_block(); return; }
    // 9/7: ScaleHTFilter (PostDecompressFilters.h:161-176) on the decoder's 32-bit sample, whose
    // magnitude LSB sits at p = 30 - k_msbs (ojph_block_decoder.cpp:1222); G.step = stepsize /
    // 2^(31 - band numbps).  k_msbs > 29 does not fit 32 bits (:1028-1030).
    const bool irrev = G.flags & 1;
    const uint32_t kmsbs = (uint32_t)G.band_numbps - (uint32_t)G.numbps;
    if (G.npasses && lcup && kmsbs > 29) { atomicOr(err, 4); zero_block(); return; }
    const uint32_t pbit = 30 - kmsbs;
    // ROI maxshift on the indices: a magnitude at or above 2^shift is the region's and scales back
    // down (standard-correct; Grok's RoiShiftHTFilter / RoiScaleHTFilter, PostDecompressFilters.h:
    // 92-158, AND the shifted magnitude with the sign bit, R-BUG-9, and are not reproduced)
    const uint32_t rshift = G.flags >> 3;
    if (!G.npasses || lcup < 2) {
        if (lcup == 1 || (G.npasses && lcup)) atomicOr(err, 4);
        zero_block();
        return;
    }
    const uint8_t* d = bytes + G.data_off;
    const uint32_t scup = ((uint32_t)d[lcup - 1] << 4) | (d[lcup - 2] & 0xF);
    if (scup < 2 || scup > lcup || scup > 4079) { atomicOr(err, 4); zero_block(); return; }
    const uint32_t pcup = lcup - scup;
    const int umax = (int)G.band_numbps - (int)G.numbps + 2;   // k_msbs + 2

    // ---- MagSgn reader: forward, LSB first, 7 bits after 0xFF, 0xFF past Pcup
    uint64_t ms_acc = 0; int ms_n = 0; bool ms_ff = false; uint32_t ms_p = 0;
    uint32_t ms_w = 0; int ms_wb = 0;
    auto ms_get = [&](int m) -> uint32_t {
        while (ms_n < m) {
            uint32_t byte;
            if (ms_p < pcup) {
                if (ms_wb == 0) { ms_w = *(const uint32_t*)(d + (ms_p & ~3u)); ms_w >>= 8 * (ms_p & 3); ms_wb = 4 - (int)(ms_p & 3); }
                byte = ms_w & 0xFF; ms_w >>= 8; --ms_wb;
            } else byte = 0xFF;
            ++ms_p;
            const int k = ms_ff ? 7 : 8;
            ms_acc |= (uint64_t)(byte & ((1u << k) - 1)) << ms_n;
            ms_n += k;
            ms_ff = byte == 0xFF;
        }
        const uint32_t v = (uint32_t)(ms_acc & ((1ull << m) - 1));
        ms_acc >>= m; ms_n -= m;
        return v;
    };
    // ---- MEL reader: forward from Pcup, MSB first, 7 bits after 0xFF
    uint32_t mel_p = pcup, mel_cur = 0; int mel_bits = 0; bool mel_ff = false;
    int mel_k = 0, mel_run = 0; bool mel_one = false;
    auto mel_bit = [&]() -> int {
        if (mel_bits == 0) {
            const uint32_t byte = mel_p < lcup ? d[mel_p] : 0xFF;
            ++mel_p;
            mel_bits = mel_ff ? 7 : 8;
            mel_cur = byte & ((1u << mel_bits) - 1);
            mel_ff = byte == 0xFF;
        }
        --mel_bits;
        return (int)((mel_cur >> mel_bits) & 1);
    };
    auto mel_event = [&]() -> int {
        if (mel_run > 0) { --mel_run; return 0; }
        if (mel_one) { mel_one = false; return 1; }
        if (mel_bit()) {
            mel_run = (1 << mel_exp(mel_k)) - 1;
            mel_k = min(12, mel_k + 1);
            return 0;
        }
        const int e = mel_exp(mel_k);
        int r = 0;
        for (int t = 0; t < e; ++t) r = (r << 1) | mel_bit();
        mel_k = max(0, mel_k - 1);
        if (r == 0) return 1;
        mel_run = r - 1; mel_one = true;
        return 0;
    };
    // ---- VLC reader: backward from Lcup-2, LSB first; the first byte holds 4 (or 3) bits
    int v_p = (int)lcup - 3; uint64_t v_acc; int v_n; bool v_gt;
    {
        const uint32_t d0 = d[lcup - 2];
        const uint32_t t = d0 >> 4;
        v_n = ((t & 7) == 7) ? 3 : 4;
        v_acc = t & ((1u << v_n) - 1);
        v_gt = d0 > 0x8F;
    }
    auto v_fill = [&]() {
        while (v_n <= 32) {
            const uint32_t byte = v_p >= (int)pcup ? d[v_p] : 0u;
            --v_p;
            const int k = (v_gt && (byte & 0x7F) == 0x7F) ? 7 : 8;
            v_acc |= (uint64_t)(byte & ((1u << k) - 1)) << v_n;
            v_n += k;
            v_gt = byte > 0x8F;
        }
    };
    auto v_get = [&](int n) -> uint32_t {
        const uint32_t v = (uint32_t)(v_acc & ((1ull << n) - 1));
        v_acc >>= n; v_n -= n;
        return v;
    };
    auto uvlc_prefix = [&]() -> int {   // 1, 2, 3 (-> 3|4) or 5 (-> 5+)
        if (v_get(1)) return 1;
        if (v_get(1)) return 2;
        return v_get(1) ? 3 : 5;
    };
    auto uvlc_suffix = [&](int pre) -> int {
        if (pre == 3) return 3 + (int)v_get(1);
        if (pre == 5) return 5 + (int)v_get(5);
        return pre;
    };

    bool bad = false;
    // one quad's samples: MagSgn values -> coefficients; returns exponents via e[]
    auto emit = [&](uint32_t x, uint32_t y, int rho, int Uq, int ek, int e1, int* e) {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const uint32_t xx = x + (n >> 1), yy = y + (n & 1);
            int32_t val = 0;
            e[n] = 0;
            if ((rho >> n) & 1) {
                const int m = Uq - ((ek >> n) & 1);
                uint32_t v = 0;
                if (m < 0 || m > 31) bad = true;
                else v = (m ? ms_get(m) : 0u) | ((uint32_t)((e1 >> n) & 1) << m);
                const uint32_t mu = (v >> 1) + 1;
                e[n] = 32 - __clz(2 * mu - 1);
                const uint32_t mo = (rshift && mu >= (1u << rshift)) ? mu >> rshift : mu;
                val = (v & 1) ? -(int32_t)mo : (int32_t)mo;
            }
            uint32_t bits = (uint32_t)val;
            if (irrev) {
                const uint32_t mag = ((uint32_t)(val < 0 ? -val : val) << pbit) & 0x7fffffffu;
                const float f = (float)mag * G.step;
                bits = __float_as_uint(val < 0 ? -f : f);
            }
            s_out[yy & 1][xx & (HT_OUTC - 1)][tid] = bits;
        }
    };
    // columns [x8, x8 + HT_OUTC) of rows y, y + 1 (those inside the block) from the staging
    auto flush = [&](uint32_t x8, uint32_t y) {
        const uint32_t nc = min((uint32_t)HT_OUTC, w - x8);
        for (uint32_t r = 0; r < 2 && y + r < h; ++r) {
            uint32_t* row = reinterpret_cast<uint32_t*>(dst + (size_t)(y + r) * stride + x8);
            if (nc == HT_OUTC && ((uintptr_t)row & 15) == 0) {
#pragma unroll
                for (uint32_t k = 0; k < HT_OUTC; k += 4)
                    reinterpret_cast<uint4*>(row)[k / 4] =
                        make_uint4(s_out[r][k][tid], s_out[r][k + 1][tid], s_out[r][k + 2][tid], s_out[r][k + 3][tid]);
            } else {
                for (uint32_t k = 0; k < nc; ++k) row[k] = s_out[r][k][tid];
            }
        }
    };

    int c_q0 = 0;
    for (uint32_t y = 0; y < h && !bad; y += 2) {
        const bool first = y == 0;
        const uint16_t* tbl = s_tab[first ? 0 : 1];
        int max_e = 0;
        if (!first) {
            max_e = max((int)s_e[0][tid], (int)s_e[1][tid]) - 1;
            s_e[0][tid] = 0;
            c_q0 = s_cx[0][tid] + (s_cx[1][tid] << 2);
            s_cx[0][tid] = 0;
        } else {
            s_e[0][tid] = 0; s_cx[0][tid] = 0;
        }
        uint32_t li = 0;
        for (uint32_t x = 0; x < w; x += 4) {
            const bool two = x + 2 < w;
            int rho[2] = {0, 0}, uoff[2] = {0, 0}, ek[2] = {0, 0}, e1[2] = {0, 0}, u[2] = {0, 0};
            v_fill();
            // quad 0: significance (MEL when the context is 0) and CxtVLC codeword
            if (c_q0 != 0 || mel_event()) {
                const uint32_t t = tbl[(c_q0 << 7) | (uint32_t)(v_acc & 0x7F)];
                v_get(t & 7);
                rho[0] = (t >> 4) & 15; uoff[0] = (t >> 3) & 1; e1[0] = (t >> 8) & 15; ek[0] = (t >> 12) & 15;
            }
            int c_q1 = first ? 0 : s_cx[li + 1][tid] + (s_cx[li + 2][tid] << 2);
            if (two) {
                if (first) c_q1 = (rho[0] >> 1) | (rho[0] & 1);
                else c_q1 |= ((rho[0] & 4) >> 1) | ((rho[0] & 8) >> 2);
                if (c_q1 != 0 || mel_event()) {
                    const uint32_t t = tbl[(c_q1 << 7) | (uint32_t)(v_acc & 0x7F)];
                    v_get(t & 7);
                    rho[1] = (t >> 4) & 15; uoff[1] = (t >> 3) & 1; e1[1] = (t >> 8) & 15; ek[1] = (t >> 12) & 15;
                }
            }
            // U-VLC exponent offsets
            if (first && uoff[0] && uoff[1]) {
                if (mel_event()) {
                    const int p0 = uvlc_prefix(), p1 = uvlc_prefix();
                    u[0] = uvlc_suffix(p0) + 2; u[1] = uvlc_suffix(p1) + 2;
                } else {
                    const int p0 = uvlc_prefix();
                    if (p0 > 2) { u[1] = (int)v_get(1) + 1; u[0] = uvlc_suffix(p0); }
                    else { const int p1 = uvlc_prefix(); u[0] = uvlc_suffix(p0); u[1] = uvlc_suffix(p1); }
                }
            } else {
                const int p0 = uoff[0] ? uvlc_prefix() : 0, p1 = uoff[1] ? uvlc_prefix() : 0;
                u[0] = uoff[0] ? uvlc_suffix(p0) : 0; u[1] = uoff[1] ? uvlc_suffix(p1) : 0;
            }
            int e[8];
            const int kappa0 = (first || !(rho[0] & (rho[0] - 1))) ? 1 : max(1, max_e);
            const int Uq0 = kappa0 + u[0];
            if (rho[0] && Uq0 > umax) bad = true;
            emit(x, y, rho[0], Uq0, ek[0], e1[0], e);
            s_e[li][tid] = (uint8_t)max((int)s_e[li][tid], e[1]);
            ++li;
            if (!first) max_e = max((int)s_e[li][tid], (int)s_e[li + 1][tid]) - 1;
            s_e[li][tid] = (uint8_t)e[3];
            s_cx[li - 1][tid] = (uint8_t)(s_cx[li - 1][tid] | ((rho[0] & 2) >> 1));
            s_cx[li][tid] = (uint8_t)((rho[0] & 8) >> 3);
            if (two) {
                const int kappa1 = (first || !(rho[1] & (rho[1] - 1))) ? 1 : max(1, max_e);
                const int Uq1 = kappa1 + u[1];
                if (rho[1] && Uq1 > umax) bad = true;
                emit(x + 2, y, rho[1], Uq1, ek[1], e1[1], e + 4);
                s_e[li][tid] = (uint8_t)max((int)s_e[li][tid], e[5]);
                ++li;
                if (!first) max_e = max((int)s_e[li][tid], (int)s_e[li + 1][tid]) - 1;
                s_e[li][tid] = (uint8_t)e[7];
                s_cx[li - 1][tid] = (uint8_t)(s_cx[li - 1][tid] | ((rho[1] & 2) >> 1));
                if (!first) c_q0 = s_cx[li][tid] + (s_cx[li + 1][tid] << 2);
                s_cx[li][tid] = (uint8_t)((rho[1] & 8) >> 3);
            }
            if (first) c_q0 = (rho[1] >> 1) | (rho[1] & 1);
            else c_q0 |= ((rho[1] & 4) >> 1) | ((rho[1] & 8) >> 2);
            if ((x & (HT_OUTC - 4)) == HT_OUTC - 4 || x + 4 >= w) flush(x & ~(uint32_t)(HT_OUTC - 1), y);
        }
        if (first) s_e[li + 1][tid] = 0;
    }
    if (bad) { atomicOr(err, 4); zero_block(); }
}

// blocks per 64-lane wave (1..64).  C4 (66,304 blocks), T1 encode / decode: 64 lanes 3.13 / 5.50
// ms, 48 lanes 3.04 / 5.17, 32 lanes 3.27 / 5.23, 16 lanes 5.38 / 8.33 (one wave per SIMD leaves
// each serial coder's memory waits exposed; 48 lanes put a second wave on a third of the SIMDs)
static uint32_t ht_lanes(const char* var) {
    const char* v = getenv(var);
    const int n = v ? atoi(v) : 48;
    return (uint32_t)(n < 1 ? 1 : (n > 64 ? 64 : n));
}
void gk_launch_ht_enc(hipStream_t st, const int32_t* coef, const GkBlock* blocks, uint8_t* bytes, uint8_t* mel_scratch,
                      uint32_t mel_cap, uint32_t* info, uint32_t nblocks, int* err, bool wide) {
    if (!nblocks) return;
    static const uint32_t nl = ht_lanes("GK_HT_ENC_LANES");
    if (wide) {
        const uint32_t per = (HT_WG_WIDE / 64) * nl;
        hipLaunchKernelGGL((k_ht_enc<HT_WG_WIDE, HT_LINE_WIDE>), dim3((nblocks + per - 1) / per), dim3(HT_WG_WIDE), 0, st,
                           coef, blocks, bytes, mel_scratch, mel_cap, info, nblocks, err, nl);
        return;
    }
    const uint32_t per = (HT_WG_STD / 64) * nl;
    hipLaunchKernelGGL((k_ht_enc<HT_WG_STD, HT_LINE_STD>), dim3((nblocks + per - 1) / per), dim3(HT_WG_STD), 0, st, coef, blocks, bytes,
                       mel_scratch, mel_cap, info, nblocks, err, nl);
}

void gk_launch_ht_dec(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, const uint32_t* ids, int32_t* coef,
                      uint32_t nblocks, int* err, bool wide) {
    if (!nblocks) return;
    static const uint32_t nl = ht_lanes("GK_HT_DEC_LANES");
    if (wide) {
        const uint32_t per = (HT_WG_WIDE / 64) * nl;
        hipLaunchKernelGGL((k_ht_dec<HT_WG_WIDE, HT_LINE_WIDE>), dim3((nblocks + per - 1) / per), dim3(HT_WG_WIDE), 0, st,
                           bytes, blocks, ids, coef, nblocks, err, nl);
        return;
    }
    const uint32_t per = (HT_WG_STD / 64) * nl;
    hipLaunchKernelGGL((k_ht_dec<HT_WG_STD, HT_LINE_STD>), dim3((nblocks + per - 1) / per), dim3(HT_WG_STD), 0, st, bytes, blocks, ids,
                       coef, nblocks, err, nl);
}
