// gk_launch.h — host-side launch wrappers for the kernels in gk_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"

// Dispatch on the caller's sample type (GkSample): T names the element type in the body.
#define GK_SAMPLE_DISPATCH(t, T, ...)                            \
    switch (t) {                                                 \
        case GK_U8: { typedef uint8_t T; __VA_ARGS__; break; }   \
        case GK_S8: { typedef int8_t T; __VA_ARGS__; break; }    \
        case GK_U16: { typedef uint16_t T; __VA_ARGS__; break; } \
        case GK_S16: { typedef int16_t T; __VA_ARGS__; break; }  \
        default: { typedef int32_t T; __VA_ARGS__; break; }      \
    }

// DC shift / MCT between the caller's planes (sample type stype, GkSample) and the int32 work planes
void gk_launch_dc_rct_fwd(hipStream_t st, int stype, const void* r, const void* g, const void* b, uint32_t sin,
                          int32_t* y, int32_t* u, int32_t* v, uint32_t sout, uint32_t w, uint32_t h, int32_t shift);
void gk_launch_dc_fwd(hipStream_t st, int stype, const void* in, uint32_t sin, int32_t* out, uint32_t sout, uint32_t w,
                      uint32_t h, int32_t shift);
void gk_launch_rct_inv_dc(hipStream_t st, const int32_t* y, const int32_t* u, const int32_t* v, uint32_t sin, int stype,
                          void* r, void* g, void* b, uint32_t sout, uint32_t w, uint32_t h, int32_t shift,
                          int32_t mn, int32_t mx);
void gk_launch_dc_inv(hipStream_t st, const int32_t* in, uint32_t sin, int stype, void* out, uint32_t sout, uint32_t w,
                      uint32_t h, int32_t shift, int32_t mn, int32_t mx);
// one DWT level of cs.n components (planes cs.cstride apart), every tile of tb
// components per workgroup of a DWT level launch (gk_kernels.hip)
uint32_t gk_dwt_cpw(uint32_t wgs, uint32_t n, bool multi);
void gk_launch_dwt53_fwd(hipStream_t st, const int32_t* src, uint32_t sstride, int32_t* dst, uint32_t dstride,
                         uint32_t w, uint32_t h, GkTiles tb = GkTiles(), GkComps cs = GkComps());
void gk_launch_dwt53_inv(hipStream_t st, const int32_t* src, uint32_t sstride, int32_t* dst, uint32_t dstride,
                         uint32_t w, uint32_t h, GkTiles tb = GkTiles(), GkComps cs = GkComps());
// level 1 fused with the sample stage: nc = 3 (DC + RCT of three components) or 1 (DC of one)
void gk_launch_dwt53_fwd_l1(hipStream_t st, int stype, int nc, GkPtr3 in, uint32_t sin, int32_t* dst, uint64_t cstride,
                            uint32_t dstride, uint32_t w, uint32_t h, GkTiles tb, int32_t shift);
void gk_launch_dwt53_inv_l1(hipStream_t st, int stype, int nc, const int32_t* src, uint64_t cstride, uint32_t sstride,
                            GkPtr3 out, uint32_t ostride, GkWin win, uint32_t w, uint32_t h, GkTiles tb, int32_t shift,
                            int32_t mn, int32_t mx);
void gk_launch_gather(hipStream_t st, const uint8_t* src, uint8_t* dst, const uint64_t* seg, uint32_t nseg);
// T1 encode of `count` blocks: positions [base, base + count) of `order` (block ids), or blocks
// [base, base + count) without one; count = ~0u: all nblocks
void gk_launch_t1_cm(hipStream_t st, const int32_t* coef, const GkBlock* blocks, const uint64_t* sym_off, uint8_t* sym,
                     uint32_t* pass_end, uint32_t* cm_info, uint32_t nblocks, int* err, const int16_t* nmse_tab,
                     int32_t* pass_nmse, const uint32_t* order = nullptr, uint32_t base = 0, uint32_t count = 0xffffffffu);
void gk_launch_t1_mq(hipStream_t st, const uint8_t* sym, const uint64_t* sym_off, const uint32_t* pass_end,
                     const uint32_t* cm_info, const GkBlock* blocks, uint8_t* bytes, GkPass* passes, uint32_t* info,
                     uint32_t nblocks, int* err, const int32_t* pass_nmse, uint32_t* pass_counter,
                     const uint32_t* order = nullptr, uint32_t base = 0, uint32_t count = 0xffffffffu,
                     uint32_t nsolo = 0);   // nsolo: the first positions coded by solo waves, one block each
// per-block coded bit-plane count (weight of the chunked CM / MQ overlap)
void gk_launch_t1_weight(hipStream_t st, const int32_t* coef, const GkBlock* blocks, uint32_t* weight, uint32_t nblocks);
uint32_t gk_t1dec_lanes();
// counters of the last k_t1_dec2 launch made with GK_T1_STATS set: max steps per wave, steps,
// symbols (lane-parallel waves), decisions of the solo waves and of the busiest one
void gk_t1dec_stats(uint64_t out[5]);
// solo waves (gk_t1dec.hip solo_block) for a decode: how many the spare SIMDs hold (a multiple
// of 12), a forced block count (one per wave; -1: the host packs), the host's cost ratio
struct GkSoloPlan { uint32_t waves; int forced; float ratio; };
GkSoloPlan gk_t1dec_solo_plan(uint32_t nblocks, uint32_t lanes);
// the first nsolo waves of `order` are solo waves (a multiple of 12)
void gk_launch_t1_dec(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, const uint32_t* order,
                      uint64_t* scratch, const uint64_t* wave_off, uint32_t nblocks, uint32_t nsolo);
void gk_launch_t1_recon(hipStream_t st, const GkBlock* blocks, const uint32_t* ids, const uint32_t* pos,
                        const uint64_t* scratch, const uint64_t* wave_off, int32_t* coef, uint32_t nblocks,
                        uint32_t maxnp);   // maxnp: the blocks' largest numbps
// one DWT level of any parity, either filter, one line per thread (gk_dwt_any.hip): forward
// reads the input region of `in` and leaves the Mallat level in `out`, inverse the reverse
void gk_launch_dwt_any(hipStream_t st, bool irrev, bool forward, int32_t* in, int32_t* out, uint32_t stride, uint32_t w,
                       uint32_t h, uint32_t px, uint32_t py, GkTiles tb, GkComps cs, bool partial = false);
// irreversible path (gk_dwt97.hip)
// code-blocks with mode switches (gk_t1ms.hip)
void gk_launch_t1_enc_ms(hipStream_t st, const int32_t* coef, const GkBlock* blocks, uint8_t* bytes, GkPass* passes,
                         uint32_t* info, uint32_t nblocks, int* err, const int16_t* nmse_tab, uint32_t* pass_counter,
                         uint8_t* state, uint32_t sty);
void gk_launch_t1_dec_ms(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, const uint32_t* seglen, int32_t* coef,
                         uint32_t nblocks, uint8_t* state, uint32_t sty);
size_t gk_t1ms_state_bytes(uint32_t nblocks);
void gk_launch_dc_ict_fwd(hipStream_t st, int stype, const void* r, const void* g, const void* b, uint32_t sin, float* y,
                          float* u, float* v, uint32_t sout, uint32_t w, uint32_t h, int32_t shift);
void gk_launch_dc_fwd_f(hipStream_t st, int stype, const void* in, uint32_t sin, float* out, uint32_t sout, uint32_t w,
                        uint32_t h, int32_t shift);
void gk_launch_ict_inv_dc(hipStream_t st, const float* y, const float* u, const float* v, uint32_t sin, int stype, void* r,
                          void* g, void* b, uint32_t sout, uint32_t w, uint32_t h, int32_t shift, int32_t mn,
                          int32_t mx);
void gk_launch_dc_inv_f(hipStream_t st, const float* in, uint32_t sin, int stype, void* out, uint32_t sout, uint32_t w,
                        uint32_t h, int32_t shift, int32_t mn, int32_t mx);
void gk_launch_dwt97_fwd(hipStream_t st, const float* src, uint32_t sstride, float* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb = GkTiles(), GkComps cs = GkComps());
void gk_launch_dwt97_inv(hipStream_t st, const float* src, uint32_t sstride, float* dst, uint32_t dstride, uint32_t w,
                         uint32_t h, GkTiles tb = GkTiles(), GkComps cs = GkComps());
// level 1 fused with the sample stage: nc = 3 (DC + ICT) or 1 (DC)
void gk_launch_dwt97_fwd_l1(hipStream_t st, int stype, int nc, GkPtr3 in, uint32_t sin, float* dst, uint64_t cstride,
                            uint32_t dstride, uint32_t w, uint32_t h, GkTiles tb, int32_t shift);
void gk_launch_dwt97_inv_l1(hipStream_t st, int stype, int nc, const float* src, uint64_t cstride, uint32_t sstride,
                            GkPtr3 out, uint32_t ostride, GkWin win, uint32_t w, uint32_t h, GkTiles tb, int32_t shift,
                            int32_t mn, int32_t mx);
// HTJ2K cleanup-pass block coder (gk_ht.hip); wide: some block is wider than 64 samples
void gk_launch_ht_enc(hipStream_t st, const int32_t* coef, const GkBlock* blocks, uint8_t* bytes, uint8_t* mel_scratch,
                      uint32_t mel_cap, uint32_t* info, uint32_t nblocks, int* err, bool wide = false);
void gk_launch_ht_dec(hipStream_t st, const uint8_t* bytes, const GkBlock* blocks, const uint32_t* ids, int32_t* coef,
                      uint32_t nblocks, int* err, bool wide = false);
