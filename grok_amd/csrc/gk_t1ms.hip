// gk_t1ms.hip — Part-1 T1 for code-blocks coded with mode switches (BYPASS/LAZY, RESET,
// TERMALL, VSC, PTERM, SEGSYM; grok.h:98-103).
//
// The streams these switches produce are the interoperability case (third-party encoders,
// Grok's `-M` option), not the throughput case: the headline path (gk_t1enc.hip /
// gk_t1dec.hip) keeps its pass-synchronous wave modelling and its lane-stepping decoder
// free of per-pass mode tests.  Here one lane walks one code-block through its passes in
// scan order (T1.cpp:498-780 encode, :934-1446 decode), with the block's state bytes
// (significance, sign, visited, refined) in a per-block scratch slab in HBM and the MQ / raw
// coder in registers:
//   k_t1_enc_ms  outputs the same per-block records as k_t1_mq (info, packed pass records,
//                bytes in the block's slot), so T2 and rate control are shared;
//   k_t1_dec_ms  decodes the codeword segments of each block (per-segment byte lengths from
//                T2, segment pass counts from T2Decompress::initSegment's rule) and writes the
//                dequantised samples into the band window like k_t1_recon.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"
#include "gk_t1_common.h"

enum { MS_LAZY = 0x01, MS_RESET = 0x02, MS_TERMALL = 0x04, MS_VSC = 0x08, MS_PTERM = 0x10, MS_SEGSYM = 0x20 };
enum { F_SIG = 1, F_NEG = 2, F_PI = 4, F_MU = 8 };
// (w + 2) x (h + 2) state bytes, rounded up: at most 1026 x 6 for the code-block shapes Grok
// accepts (4 <= w, h <= 1024, w * h <= 4096; grk_compress.cpp:981-988)
#define MS_STATE_BYTES 6208u
#define MS_CT_INIT 0xDEADBEEFu // BYPASS_CT_INIT (mqc_inl.h:24): no raw bit written yet

// Block state with a one-sample border; VSC: the last row of a stripe sees the next
// stripe's samples as insignificant (update_flags, T1.cpp:209-232).
struct MsState {
    uint8_t* s;
    uint32_t sw;
    bool vsc;
    __device__ uint8_t get(int x, int y) const { return s[(y + 1) * sw + (x + 1)]; }
    __device__ void set(int x, int y, uint8_t v) { s[(y + 1) * sw + (x + 1)] = v; }
    __device__ uint32_t nbr(int x, int y, int yc) const {
        return (vsc && y == yc + 1 && (yc & 3) == 3) ? 0u : (uint32_t)get(x, y);
    }
    // zc_rule neighbourhood: bit0 NW bit1 N bit2 NE bit3 W bit5 E bit6 SW bit7 S bit8 SE
    __device__ uint32_t zc_pat(int x, int y) const {
        auto g = [&](int xx, int yy) { return nbr(xx, yy, y) & F_SIG; };
        return g(x - 1, y - 1) | (g(x, y - 1) << 1) | (g(x + 1, y - 1) << 2) | (g(x - 1, y) << 3) |
               (g(x + 1, y) << 5) | (g(x - 1, y + 1) << 6) | (g(x, y + 1) << 7) | (g(x + 1, y + 1) << 8);
    }
    // sc_rule index: bit0 W-neg bit1 W-sig bit2 E-neg bit3 E-sig bit4 N-neg bit5 N-sig bit6 S-neg bit7 S-sig
    __device__ uint32_t sc_pat(int x, int y) const {
        auto g = [&](int xx, int yy) {
            const uint32_t v = nbr(xx, yy, y);
            return (v & F_SIG) ? (2u | ((v >> 1) & 1u)) : 0u;
        };
        return g(x - 1, y) | (g(x + 1, y) << 2) | (g(x, y - 1) << 4) | (g(x, y + 1) << 6);
    }
};

struct MsCtx {
    uint8_t st[19], mps[19];
    __device__ void reset() {   // mqc_resetstates: UNI = 46, AGG = 3, ZC0 = 4, others 0
        for (int i = 0; i < 19; ++i) { st[i] = 0; mps[i] = 0; }
        st[CTX_UNI] = 46; st[CTX_AGG] = 3; st[CTX_ZC] = 4;
    }
};

// ---------------------------------------------------------------------------------------
// Encoder (T1::compress_cblk, T1.cpp:781-932; MQ and raw coder mqc_enc.cpp:86-330)
// ---------------------------------------------------------------------------------------
struct MsEnc {
    uint32_t a, c, ct;
    int64_t bp;              // MQ: last byte written; raw: next byte to write
    uint8_t* out;
    uint32_t cap;
    uint32_t pad1, pad2;     // bytes at index -1 / -2 (the coder's left pad, zero)
    bool ovf;
    MsCtx cx;
    __device__ uint32_t B(int64_t i) const {
        if (i >= 0) return i < (int64_t)cap ? out[i] : 0u;
        return i == -1 ? pad1 : pad2;
    }
    __device__ void Bset(int64_t i, uint32_t v) {
        if (i >= 0) { if (i < (int64_t)cap) out[i] = (uint8_t)v; else ovf = true; }
        else if (i == -1) pad1 = v & 0xff; else pad2 = v & 0xff;
    }
    __device__ void byteout() {
        if (B(bp) == 0xff) { ++bp; Bset(bp, c >> 20); c &= 0xfffff; ct = 7; }
        else if ((c & 0x8000000) == 0) { ++bp; Bset(bp, c >> 19); c &= 0x7ffff; ct = 8; }
        else {
            Bset(bp, B(bp) + 1);
            if (B(bp) == 0xff) { c &= 0x7ffffff; ++bp; Bset(bp, c >> 20); c &= 0xfffff; ct = 7; }
            else { ++bp; Bset(bp, c >> 19); c &= 0x7ffff; ct = 8; }
        }
    }
    __device__ void renorm() { do { a <<= 1; c <<= 1; if (--ct == 0) byteout(); } while ((a & 0x8000) == 0); }
    __device__ void encode(int k, uint32_t d) {
        const uint32_t e = c_mq[cx.st[k]];
        const uint32_t qe = e & 0xffff;
        if (cx.mps[k] == d) {
            a -= qe;
            if ((a & 0x8000) == 0) {
                if (a < qe) a = qe; else c += qe;
                cx.st[k] = (e >> 16) & 0x3f; renorm();
            } else c += qe;
        } else {
            a -= qe;
            if (a < qe) c += qe; else a = qe;
            if ((e >> 28) & 1) cx.mps[k] ^= 1;
            cx.st[k] = (e >> 22) & 0x3f; renorm();
        }
    }
    __device__ void flush() {
        const uint32_t tempc = c + a;
        c |= 0xffff;
        if (c >= tempc) c -= 0x8000;
        c <<= ct; byteout();
        c <<= ct; byteout();
        if (B(bp) != 0xff) ++bp;
    }
    __device__ void bypass_init() { c = 0; ct = MS_CT_INIT; }
    __device__ void bypass_encode(uint32_t d) {
        if (ct == MS_CT_INIT) ct = 8;
        --ct;
        c += d << ct;
        if (ct == 0) {
            Bset(bp, c);
            ct = (B(bp) == 0xff) ? 7 : 8;
            ++bp; c = 0;
        }
    }
    __device__ uint32_t bypass_extra_bytes(bool erterm) const {
        return (ct < 7 || (ct == 7 && (erterm || B(bp - 1) != 0xff))) ? 2u : 1u;
    }
    __device__ void bypass_flush(bool erterm) {
        if (ct < 7 || (ct == 7 && (erterm || B(bp - 1) != 0xff))) {
            uint32_t bit = 0;
            while (ct > 0) { --ct; c += bit << ct; bit = 1 - bit; }
            Bset(bp, c);
            ++bp;
        } else if (ct == 7 && B(bp - 1) == 0xff) {
            --bp;
        } else if (ct == 8 && !erterm && B(bp - 1) == 0x7f && B(bp - 2) == 0xff) {
            bp -= 2;
        }
    }
    __device__ void restart_init() {
        a = 0x8000; c = 0; ct = 12;
        --bp;
        if (B(bp) == 0xff) ct = 13;
    }
    __device__ void erterm() {
        int32_t k = (int32_t)(11 - ct + 1);
        while (k > 0) { c <<= ct; ct = 0; byteout(); k -= (int32_t)ct; }
        if (B(bp) != 0xff) byteout();
    }
};

__device__ __forceinline__ bool ms_term_pass(uint32_t sty, int numbps, int bpno, int passtype) {   // T1.cpp:437-458
    if (passtype == 2 && bpno == 0) return true;
    if (sty & MS_TERMALL) return true;
    if (sty & MS_LAZY) {
        if (bpno == numbps - 4 && passtype == 2) return true;
        if (bpno < numbps - 4 && passtype > 0) return true;
    }
    return false;
}

// Lane = code-block.  state: MS_STATE_BYTES per block slot of this launch (lane index).
__global__ __launch_bounds__(64) void k_t1_enc_ms(const int32_t* __restrict__ coef, const GkBlock* __restrict__ blocks,
                                                  uint8_t* __restrict__ bytes, GkPass* __restrict__ passes,
                                                  uint32_t* __restrict__ info, uint32_t nblocks, int* err,
                                                  const int16_t* __restrict__ nmse_tab, uint32_t* __restrict__ pass_counter,
                                                  uint8_t* __restrict__ state, uint32_t sty) {
    const uint32_t b = blockIdx.x * 64 + threadIdx.x;
    if (b >= nblocks) return;
    const GkBlock G = blocks[b];
    const int w = G.w, h = G.h;
    const bool irrev = G.flags & 1, rc = (G.flags & 2) != 0;
    auto smr = [&](int x, int y) -> int32_t {   // T1Part1::preCompress (T1Part1.cpp:36-87)
        const int32_t raw = coef[G.band_off + (size_t)y * G.stride + x];
        const int32_t v = irrev ? (int32_t)rintf((__int_as_float(raw) / G.step) * 64.0f) : raw * 64;
        if (!(G.flags >> 3)) return v;
        // ROI maxshift (the component is the region): the index's integer part scaled up
        const uint32_t a0 = (uint32_t)(v < 0 ? -v : v), a1 = ((a0 >> 6) << (6 + (G.flags >> 3))) | (a0 & 63u);
        return v < 0 ? -(int32_t)a1 : (int32_t)a1;
    };
    uint32_t mx = 0;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) { const int32_t v = smr(x, y); const uint32_t m = (uint32_t)(v < 0 ? -v : v); mx = m > mx ? m : mx; }
    uint32_t numbps = 0;
    if (mx) { const uint32_t t = 32 - __clz(mx); numbps = t <= 6 ? 0 : t - 6; }
    if (numbps == 0) { info[4 * b] = 0; info[4 * b + 1] = 0; info[4 * b + 2] = 0; info[4 * b + 3] = 0; return; }
    const uint32_t npasses = 3 * numbps - 2;
    if (npasses > GK_MAX_PASSES) { atomicOr(err, 1); return; }
    const uint32_t poff = atomicAdd(pass_counter, npasses);
    GkPass* P = passes + poff;
    MsState S;
    S.s = state + (size_t)b * MS_STATE_BYTES; S.sw = (uint32_t)w + 2; S.vsc = (sty & MS_VSC) != 0;
    for (uint32_t i = 0; i < (uint32_t)(w + 2) * (uint32_t)(h + 2); ++i) S.s[i] = 0;
    MsEnc q;
    q.a = 0x8000; q.c = 0; q.ct = 12; q.bp = -1; q.out = bytes + G.data_off; q.cap = G.data_cap;
    q.pad1 = q.pad2 = 0; q.ovf = false;
    q.cx.reset();
    const int nbp = (int)numbps;
    int bpno = nbp - 1, passtype = 2;
    double cum = 0.0;
    bool prev_term = false;
    for (uint32_t passno = 0; bpno >= 0; ++passno) {
        const uint32_t one = 1u << (bpno + 6);
        int32_t nmsedec = 0;
        const bool raw = (sty & MS_LAZY) && bpno < nbp - 4 && passtype < 2;
        if (passno > 0 && prev_term) { if (raw) q.bypass_init(); else q.restart_init(); }
        auto code = [&](int k, uint32_t d) { if (raw) q.bypass_encode(d); else q.encode(k, d); };
        auto nm = [&](int t, uint32_t m) {   // getnmsedec_sig / _ref (T1.cpp:190-208)
            if (rc) nmsedec += bpno > 0 ? nmse_tab[t * 128 + ((m >> bpno) & 127)] : nmse_tab[(t + 1) * 128 + (m & 127)];
        };
        if (passtype == 0) {
            for (int k = 0; k < h; k += 4)
                for (int x = 0; x < w; ++x)
                    for (int y = k; y < min(k + 4, h); ++y) {
                        const uint8_t st = S.get(x, y);
                        if (st & (F_SIG | F_PI)) continue;
                        const uint32_t zp = S.zc_pat(x, y);
                        if (!zp) continue;
                        const int32_t v0 = smr(x, y);
                        const uint32_t m = (uint32_t)(v0 < 0 ? -v0 : v0);
                        const uint32_t v = (m & one) ? 1u : 0u;
                        code(CTX_ZC + zc_rule(G.orient, zp), v);
                        uint8_t ns = st | F_PI;
                        if (v) {
                            const uint32_t sc = sc_rule(S.sc_pat(x, y));
                            const uint32_t sg = v0 < 0;
                            nm(0, m);
                            code(CTX_SC + (sc & 15), raw ? sg : (sg ^ (sc >> 4)));
                            ns |= F_SIG | (sg ? F_NEG : 0);
                        }
                        S.set(x, y, ns);
                    }
        } else if (passtype == 1) {
            for (int k = 0; k < h; k += 4)
                for (int x = 0; x < w; ++x)
                    for (int y = k; y < min(k + 4, h); ++y) {
                        const uint8_t st = S.get(x, y);
                        if ((st & (F_SIG | F_PI)) != F_SIG) continue;
                        const int ctx = (st & F_MU) ? 2 : (S.zc_pat(x, y) ? 1 : 0);
                        const int32_t v0 = smr(x, y);
                        const uint32_t m = (uint32_t)(v0 < 0 ? -v0 : v0);
                        nm(2, m);
                        code(CTX_MAG + ctx, (m & one) ? 1u : 0u);
                        S.set(x, y, st | F_MU);
                    }
        } else {
            for (int k = 0; k < h; k += 4)
                for (int x = 0; x < w; ++x) {
                    const int ylim = min(k + 4, h);
                    int y = k;
                    if (ylim - k == 4) {
                        bool agg = true;
                        for (int yy = k; yy < ylim && agg; ++yy) {
                            if (S.get(x, yy) & (F_SIG | F_PI | F_MU)) agg = false;
                            else if (S.zc_pat(x, yy)) agg = false;
                        }
                        if (agg) {
                            int run = 0;
                            for (; run < 4; ++run) {
                                const int32_t v0 = smr(x, k + run);
                                if ((uint32_t)(v0 < 0 ? -v0 : v0) & one) break;
                            }
                            q.encode(CTX_AGG, run != 4);
                            if (run == 4) continue;
                            q.encode(CTX_UNI, (uint32_t)run >> 1);
                            q.encode(CTX_UNI, (uint32_t)run & 1);
                            y = k + run;
                            const int32_t v0 = smr(x, y);
                            const uint32_t sc = sc_rule(S.sc_pat(x, y));
                            const uint32_t sg = v0 < 0;
                            nm(0, (uint32_t)(v0 < 0 ? -v0 : v0));
                            q.encode(CTX_SC + (sc & 15), sg ^ (sc >> 4));
                            S.set(x, y, S.get(x, y) | F_SIG | (sg ? F_NEG : 0));
                            ++y;
                        }
                    }
                    for (; y < ylim; ++y) {
                        const uint8_t st = S.get(x, y);
                        if (st & (F_SIG | F_PI)) continue;
                        const int32_t v0 = smr(x, y);
                        const uint32_t m = (uint32_t)(v0 < 0 ? -v0 : v0);
                        const uint32_t v = (m & one) ? 1u : 0u;
                        q.encode(CTX_ZC + zc_rule(G.orient, S.zc_pat(x, y)), v);
                        if (v) {
                            const uint32_t sc = sc_rule(S.sc_pat(x, y));
                            const uint32_t sg = v0 < 0;
                            nm(0, m);
                            q.encode(CTX_SC + (sc & 15), sg ^ (sc >> 4));
                            S.set(x, y, st | F_SIG | (sg ? F_NEG : 0));
                        }
                    }
                    for (int yy = k; yy < ylim; ++yy) S.set(x, yy, S.get(x, yy) & (uint8_t)~F_PI);
                }
            if (sty & MS_SEGSYM)   // mqc_segmark_enc: 1, 0, 1, 0 in the UNIFORM context
                for (uint32_t i = 1; i < 5; ++i) q.encode(CTX_UNI, i & 1);
        }
        if (rc) {   // T1::getwmsedec with Grok's roundings (no fused multiply-add)
            double wm = __dmul_rn(G.wmse, (double)(1 << bpno));
            wm = __dmul_rn(wm, __dmul_rn(wm, (double)nmsedec) / 8192.0);
            cum = __dadd_rn(cum, wm);
        }
        P[passno].dist = cum;
        prev_term = ms_term_pass(sty, nbp, bpno, passtype);
        if (prev_term) {
            if (raw) q.bypass_flush((sty & MS_PTERM) != 0);
            else if (sty & MS_PTERM) q.erterm();
            else q.flush();
            P[passno].rate = (uint32_t)q.bp;
        } else {
            uint32_t extra;
            if (raw) extra = q.bypass_extra_bytes((sty & MS_PTERM) != 0);
            else extra = 5 + (q.ct < 5 ? 1 : 0);
            P[passno].rate = (uint32_t)q.bp + extra;
        }
        if (++passtype == 3) { passtype = 0; --bpno; }
        if (sty & MS_RESET) q.cx.reset();
    }
    const uint32_t nbytes = (uint32_t)q.bp;
    uint32_t last = nbytes;
    for (int k = (int)npasses; k > 0;) {   // monotone rates (T1.cpp:907-919)
        GkPass& ps = P[--k];
        if (ps.rate > last) ps.rate = last; else last = ps.rate;
    }
    uint32_t prev = 0;
    for (uint32_t k = 0; k < npasses; ++k) {   // FF back-off (T1.cpp:920-930)
        GkPass& ps = P[k];
        if (ps.rate > 0 && q.B((int64_t)ps.rate - 1) == 0xff) ps.rate--;
        ps.len = ps.rate - prev;
        prev = ps.rate;
    }
    info[4 * b] = numbps;
    info[4 * b + 1] = npasses;
    info[4 * b + 2] = P[npasses - 1].rate;
    info[4 * b + 3] = poff;
    if (q.ovf || nbytes > q.cap) atomicOr(err, 1);
}

// ---------------------------------------------------------------------------------------
// Decoder (T1::decompress_cblk, T1.cpp:1365-1446; MQ decoder mqc_dec.cpp:78-130, raw
// decoder mqc_dec_inl.h:61-91).  Bytes past a segment read as 0xFF (the artificial end
// marker mqc_init_dec_common inserts after each segment).
// ---------------------------------------------------------------------------------------
struct MsDec {
    const uint8_t* buf;
    uint32_t len, bp, a, c, ct;
    MsCtx cx;
    __device__ uint32_t at(uint32_t i) const { return i < len ? buf[i] : 0xffu; }
    __device__ void bytein() {
        const uint32_t l_c = at(bp + 1);
        if (at(bp) == 0xff) {
            if (l_c > 0x8f) { c += 0xff00; ct = 8; }
            else { ++bp; c += l_c << 9; ct = 7; }
        } else { ++bp; c += l_c << 8; ct = 8; }
    }
    __device__ void init(const uint8_t* b, uint32_t n) {
        buf = b; len = n; bp = 0;
        c = (n == 0 ? 0xffu : at(0)) << 16;
        bytein();
        c <<= 7; ct -= 7; a = 0x8000;
    }
    __device__ void raw_init(const uint8_t* b, uint32_t n) { buf = b; len = n; bp = 0; c = 0; ct = 0; }
    __device__ uint32_t raw_decode() {
        if (ct == 0) {
            if (c == 0xff) {
                if (at(bp) > 0x8f) { c = 0xff; ct = 8; }
                else { c = at(bp); ++bp; ct = 7; }
            } else { c = at(bp); ++bp; ct = 8; }
        }
        --ct;
        return (c >> ct) & 1u;
    }
    __device__ void renorm() { do { if (ct == 0) bytein(); a <<= 1; c <<= 1; --ct; } while (a < 0x8000); }
    __device__ uint32_t decode(int k) {
        const uint32_t e = c_mq[cx.st[k]];
        const uint32_t qe = e & 0xffff;
        uint32_t d;
        a -= qe;
        if (c < (qe << 16)) {
            if (a < qe) { a = qe; d = cx.mps[k]; cx.st[k] = (e >> 16) & 0x3f; }
            else { a = qe; d = cx.mps[k] ^ 1; if ((e >> 28) & 1) cx.mps[k] ^= 1; cx.st[k] = (e >> 22) & 0x3f; }
            renorm();
        } else {
            c -= qe << 16;
            if (a < 0x8000) {
                if (a < qe) { d = cx.mps[k] ^ 1; if ((e >> 28) & 1) cx.mps[k] ^= 1; cx.st[k] = (e >> 22) & 0x3f; }
                else { d = cx.mps[k]; cx.st[k] = (e >> 16) & 0x3f; }
                renorm();
            } else d = cx.mps[k];
        }
        return d;
    }
};

// Passes of codeword segment s (T2Decompress::initSegment, T2Decompress.cpp:28-54)
__device__ __forceinline__ uint32_t ms_seg_maxpasses(uint32_t sty, uint32_t s) {
    if (sty & MS_TERMALL) return 1;
    if (sty & MS_LAZY) return s == 0 ? 10 : ((s & 1) ? 2 : 1);
    return 0xffffffffu;
}

// Block b's segments: seglen[G.data_cap ...] (data_cap carries the segment-table offset on
// decode).  Output: dequantised samples in the band window (ShiftFilter / ScaleFilter,
// PostDecompressFilters.h:31-177), the decoder's 2x values staged in place first.
__global__ __launch_bounds__(64) void k_t1_dec_ms(const uint8_t* __restrict__ bytes, const GkBlock* __restrict__ blocks,
                                                  const uint32_t* __restrict__ seglen, int32_t* __restrict__ coef,
                                                  uint32_t nblocks, uint8_t* __restrict__ state, uint32_t sty) {
    const uint32_t b = blockIdx.x * 64 + threadIdx.x;
    if (b >= nblocks) return;
    const GkBlock G = blocks[b];
    const int w = G.w, h = G.h;
    int32_t* o = coef + G.band_off;
    const uint32_t os = G.stride;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) o[(size_t)y * os + x] = 0;
    const uint32_t numbps = G.numbps, npasses = G.npasses;
    if (npasses && numbps) {
        MsState S;
        S.s = state + (size_t)b * MS_STATE_BYTES; S.sw = (uint32_t)w + 2; S.vsc = (sty & MS_VSC) != 0;
        for (uint32_t i = 0; i < (uint32_t)(w + 2) * (uint32_t)(h + 2); ++i) S.s[i] = 0;
        const uint8_t* data = bytes + G.data_off;
        const uint32_t len = G.len;
        MsDec q;
        q.cx.reset();
        int bpno1 = (int)numbps, passtype = 2;
        uint32_t segno = 0, off = 0, seg_left = 0;
        bool raw = false;
        for (uint32_t p = 0; p < npasses && bpno1 >= 1; ++p) {
            if (seg_left == 0) {
                const uint32_t sl = seglen ? seglen[G.data_cap + segno] : len;   // no table: one segment
                const uint32_t sb = min(sl, len - min(off, len));
                raw = (sty & MS_LAZY) && bpno1 <= (int)numbps - 4 && passtype < 2;
                if (raw) q.raw_init(data + off, sb); else q.init(data + off, sb);
                off += sb;
                seg_left = ms_seg_maxpasses(sty, segno++);
            }
            --seg_left;
            const int32_t one = 1 << bpno1, half = one >> 1, oph = one | half;
            if (passtype == 0) {
                for (int k = 0; k < h; k += 4)
                    for (int x = 0; x < w; ++x)
                        for (int y = k; y < min(k + 4, h); ++y) {
                            const uint8_t st = S.get(x, y);
                            if (st & (F_SIG | F_PI)) continue;
                            const uint32_t zp = S.zc_pat(x, y);
                            if (!zp) continue;
                            uint8_t ns = st | F_PI;
                            if (raw ? q.raw_decode() : q.decode(CTX_ZC + zc_rule(G.orient, zp))) {
                                const uint32_t sc = sc_rule(S.sc_pat(x, y));
                                const uint32_t sg = raw ? q.raw_decode() : (q.decode(CTX_SC + (sc & 15)) ^ (sc >> 4));
                                o[(size_t)y * os + x] = sg ? -oph : oph;
                                ns |= F_SIG | (sg ? F_NEG : 0);
                            }
                            S.set(x, y, ns);
                        }
            } else if (passtype == 1) {
                for (int k = 0; k < h; k += 4)
                    for (int x = 0; x < w; ++x)
                        for (int y = k; y < min(k + 4, h); ++y) {
                            const uint8_t st = S.get(x, y);
                            if ((st & (F_SIG | F_PI)) != F_SIG) continue;
                            const int ctx = (st & F_MU) ? 2 : (S.zc_pat(x, y) ? 1 : 0);
                            const uint32_t v = raw ? q.raw_decode() : q.decode(CTX_MAG + ctx);
                            int32_t& d = o[(size_t)y * os + x];
                            d += (v ^ (d < 0 ? 1u : 0u)) ? half : -half;
                            S.set(x, y, st | F_MU);
                        }
            } else {
                for (int k = 0; k < h; k += 4)
                    for (int x = 0; x < w; ++x) {
                        const int ylim = min(k + 4, h);
                        int y = k;
                        bool partial = false;
                        if (ylim - k == 4) {
                            bool agg = true;
                            for (int yy = k; yy < ylim && agg; ++yy) {
                                if (S.get(x, yy) & (F_SIG | F_PI | F_MU)) agg = false;
                                else if (S.zc_pat(x, yy)) agg = false;
                            }
                            if (agg) {
                                if (!q.decode(CTX_AGG)) continue;
                                uint32_t r = q.decode(CTX_UNI);
                                r = (r << 1) | q.decode(CTX_UNI);
                                y = k + (int)r;
                                partial = true;
                            }
                        }
                        for (; y < ylim; ++y) {
                            const uint8_t st = S.get(x, y);
                            if (!partial) {
                                if (st & (F_SIG | F_PI)) continue;
                                if (!q.decode(CTX_ZC + zc_rule(G.orient, S.zc_pat(x, y)))) continue;
                            }
                            partial = false;
                            const uint32_t sc = sc_rule(S.sc_pat(x, y));
                            const uint32_t sg = q.decode(CTX_SC + (sc & 15)) ^ (sc >> 4);
                            o[(size_t)y * os + x] = sg ? -oph : oph;
                            S.set(x, y, st | F_SIG | (sg ? F_NEG : 0));
                        }
                        for (int yy = k; yy < ylim; ++yy) S.set(x, yy, S.get(x, yy) & (uint8_t)~F_PI);
                    }
                if (sty & MS_SEGSYM)   // dec_clnpass_check_segsym: four UNIFORM decisions
                    for (int i = 0; i < 4; ++i) q.decode(CTX_UNI);
            }
            if ((sty & MS_RESET) && !raw) q.cx.reset();
            if (++passtype == 3) { passtype = 0; --bpno1; }
        }
    }
    const bool irrev = G.flags & 1;
    const uint32_t rs = G.flags >> 3;   // ROI shift (RoiShiftFilter / RoiScaleFilter)
    float* fo = reinterpret_cast<float*>(o);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const size_t i = (size_t)y * os + x;
            int32_t v = o[i];
            if (rs) {
                const int32_t m = v < 0 ? -v : v;
                if (m >= (1 << rs)) v = v < 0 ? -(m >> rs) : (m >> rs);
            }
            if (irrev) fo[i] = (float)v * G.step;
            else o[i] = v / 2;
        }
}

#include "gk_launch.h"
void gk_launch_t1_enc_ms(hipStream_t st, const int32_t* coef, const GkBlock* blocks, uint8_t* bytes, GkPass* passes,
                         uint32_t* info, uint32_t nblocks, int* err, const int16_t* nmse_tab, uint32_t* pass_counter,
                         uint8_t* state, uint32_t sty) {
    if (!nblocks) return;
    hipLaunchKernelGGL(k_t1_enc_ms, dim3((nblocks + 63) / 64), dim3(64), 0, st, coef, blocks, bytes, passes, info, nblocks,
                       err, nmse_tab, pass_counter, state, sty);
}
void gk_launch_t1_dec_ms(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, const uint32_t* seglen, int32_t* coef,
                         uint32_t nblocks, uint8_t* state, uint32_t sty) {
    if (!nblocks) return;
    hipLaunchKernelGGL(k_t1_dec_ms, dim3((nblocks + 63) / 64), dim3(64), 0, st, bytes, blocks, seglen, coef, nblocks, state,
                       sty);
}
size_t gk_t1ms_state_bytes(uint32_t nblocks) { return (size_t)nblocks * MS_STATE_BYTES; }
