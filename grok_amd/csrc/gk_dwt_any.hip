// gk_dwt_any.hip — DWT levels of any parity (5/3 and 9/7), one line per thread.
//
// A resolution whose origin lies on an odd coordinate (tile sizes off the 2^L grid, e.g.
// grk_compress -t 200,160) starts with a high-pass sample: WaveletFwd.cpp picks the odd
// ("cas1") lifting from parity_row / parity_col (:486-489) and WaveletReverse.cpp:559-663 its
// inverse.  The LDS-tiled kernels (gk_kernels.hip, gk_dwt97.hip) take parity 0, which every
// tile of a 2^L-aligned grid has; tile classes with an odd parity at some level run these
// kernels for that level instead.  They follow the restated line transforms exactly: sample i
// of a line is high-pass when (i + parity) is odd, whole-sample symmetric extension at both
// ends, lows then highs on output; a single sample is doubled (5/3 forward, odd parity) or
// halved (5/3 inverse: bandH / 2 across, bandL >> 1 down, WaveletReverse.cpp:583, :636; a
// windowed decode takes Grok's partial-tile path, whose horizontal case shifts too,
// S(buf, 0) >>= 1 at :1551-1554, and differs from / 2 for a negative odd coefficient) and
// left as it is by the 9/7.  9/7 steps are rounded one operation at a time (no contraction),
// as the tiled kernels and Grok's scalar path do.
//
// Forward level (vertical first, as WaveletFwd.cpp): columns are lifted in place in the level's
// input region and written deinterleaved to the output plane; rows are lifted there in place
// and written deinterleaved back to the input region, which is then copied to the output
// plane.  Inverse (horizontal first): rows are interleaved from the Mallat input into the
// output region and lifted there, columns interleaved back into the input plane and lifted,
// and the result copied to the output region.  The level's input region is only scratch once
// it is read (no other band lives in it), so no extra buffer is needed.  Lines run one per
// thread: these launches are for the tile classes an unaligned grid adds, not the fast path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"

// every 9/7 step rounds its product and its sum separately (an FMA would round once; the
// __f*_rn helpers do not stop the contraction once inlined, the pragma does)
#pragma clang fp contract(off)

namespace {
constexpr float A97 = -1.586134342f, B97 = -0.052980118f, G97 = 0.882911075f, D97 = 0.443506852f;
constexpr float K97 = 1.230174105f, INVK97 = (float)(1.0 / 1.230174105), TWO_INVK97 = 1.625732422f;

__device__ __forceinline__ int mir(int i, int n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
    return i;
}

// forward lifting in place on a line of n samples (element stride s)
__device__ void fwd53_line(int32_t* x, size_t s, int n, int par) {
    if (n == 1) { if (par) x[0] *= 2; return; }
    for (int i = 1 - par; i < n; i += 2) x[i * s] -= (x[mir(i - 1, n) * s] + x[mir(i + 1, n) * s]) >> 1;
    for (int i = par; i < n; i += 2) x[i * s] += (x[mir(i - 1, n) * s] + x[mir(i + 1, n) * s] + 2) >> 2;
}
__device__ void fwd97_line(float* x, size_t s, int n, int par) {
    if (n < 2) return;
    auto step = [&](int start, float c) {
        for (int i = start; i < n; i += 2) {
            const float t = (x[mir(i - 1, n) * s] + x[mir(i + 1, n) * s]) * c;
            x[i * s] = x[i * s] + t;
        }
    };
    step(1 - par, A97); step(par, B97); step(1 - par, G97); step(par, D97);
}
// lows then highs of line x into line y (9/7: lows x 1/K, highs x K unless a single sample)
template <bool IRREV, class T>
__device__ void deinterleave(const T* x, size_t sx, T* y, size_t sy, int n, int par) {
    int k = 0;
    for (int i = par; i < n; i += 2, ++k) {
        T v = x[i * sx];
        if constexpr (IRREV) if (n > 1) v = v * INVK97;
        y[k * sy] = v;
    }
    for (int i = 1 - par; i < n; i += 2, ++k) {
        T v = x[i * sx];
        if constexpr (IRREV) if (n > 1) v = v * K97;
        y[k * sy] = v;
    }
}
// Mallat line x (lows then highs) interleaved into line y, then inverse lifting in place
__device__ void inv53_line(const int32_t* x, size_t sx, int32_t* y, size_t sy, int n, int par, bool shift) {
    if (n == 1) {
        int32_t v = x[0];
        if (par) v = shift ? (v >> 1) : (v / 2);
        y[0] = v;
        return;
    }
    int k = 0;
    for (int i = par; i < n; i += 2) y[i * sy] = x[(k++) * sx];
    for (int i = 1 - par; i < n; i += 2) y[i * sy] = x[(k++) * sx];
    for (int i = par; i < n; i += 2) y[i * sy] -= (y[mir(i - 1, n) * sy] + y[mir(i + 1, n) * sy] + 2) >> 2;
    for (int i = 1 - par; i < n; i += 2) y[i * sy] += (y[mir(i - 1, n) * sy] + y[mir(i + 1, n) * sy]) >> 1;
}
__device__ void inv97_line(const float* x, size_t sx, float* y, size_t sy, int n, int par) {
    if (n < 2) { if (n == 1) y[0] = x[0]; return; }
    int k = 0;
    for (int i = par; i < n; i += 2) y[i * sy] = x[(k++) * sx] * K97;
    for (int i = 1 - par; i < n; i += 2) y[i * sy] = x[(k++) * sx] * TWO_INVK97;
    auto step = [&](int start, float c) {
        for (int i = start; i < n; i += 2) {
            const float t = c * (y[mir(i - 1, n) * sy] + y[mir(i + 1, n) * sy]);
            y[i * sy] = y[i * sy] - t;
        }
    };
    step(par, D97); step(1 - par, G97); step(par, B97); step(1 - par, A97);
}

struct AnyLevel {
    uint32_t w, h, px, py;
    uint32_t partial;   // a windowed decode (Grok's partial-tile inverse)
    GkTiles tb;
    uint64_t cstride;
    uint32_t stride;
};
// line `line` of tile-component z (blockIdx.y): the tile's region offset in its component plane
__device__ __forceinline__ uint64_t region(const AnyLevel& a, uint32_t z) {
    const uint32_t nt = a.tb.count();
    return (uint64_t)(z / nt) * a.cstride + a.tb.offset(z % nt, a.stride);
}

template <bool IRREV>
__global__ __launch_bounds__(64) void k_any_fwd_cols(int32_t* src, int32_t* dst, AnyLevel a) {
    const uint32_t x = blockIdx.x * 64 + threadIdx.x;
    if (x >= a.w) return;
    const uint64_t o = region(a, blockIdx.y) + x;
    if constexpr (IRREV) {
        float* s = reinterpret_cast<float*>(src) + o;
        fwd97_line(s, a.stride, (int)a.h, (int)a.py);
        deinterleave<true>(s, a.stride, reinterpret_cast<float*>(dst) + o, a.stride, (int)a.h, (int)a.py);
    } else {
        fwd53_line(src + o, a.stride, (int)a.h, (int)a.py);
        deinterleave<false>(src + o, a.stride, dst + o, a.stride, (int)a.h, (int)a.py);
    }
}
template <bool IRREV>
__global__ __launch_bounds__(64) void k_any_fwd_rows(int32_t* src, int32_t* dst, AnyLevel a) {
    const uint32_t y = blockIdx.x * 64 + threadIdx.x;
    if (y >= a.h) return;
    const uint64_t o = region(a, blockIdx.y) + (uint64_t)y * a.stride;
    if constexpr (IRREV) {
        float* d = reinterpret_cast<float*>(dst) + o;
        fwd97_line(d, 1, (int)a.w, (int)a.px);
        deinterleave<true>(d, 1, reinterpret_cast<float*>(src) + o, 1, (int)a.w, (int)a.px);
    } else {
        fwd53_line(dst + o, 1, (int)a.w, (int)a.px);
        deinterleave<false>(dst + o, 1, src + o, 1, (int)a.w, (int)a.px);
    }
}
template <bool IRREV>
__global__ __launch_bounds__(64) void k_any_inv_rows(int32_t* src, int32_t* dst, AnyLevel a) {
    const uint32_t y = blockIdx.x * 64 + threadIdx.x;
    if (y >= a.h) return;
    const uint64_t o = region(a, blockIdx.y) + (uint64_t)y * a.stride;
    if constexpr (IRREV)
        inv97_line(reinterpret_cast<const float*>(src) + o, 1, reinterpret_cast<float*>(dst) + o, 1, (int)a.w, (int)a.px);
    else
        inv53_line(src + o, 1, dst + o, 1, (int)a.w, (int)a.px, a.partial != 0);
}
template <bool IRREV>
__global__ __launch_bounds__(64) void k_any_inv_cols(int32_t* src, int32_t* dst, AnyLevel a) {
    const uint32_t x = blockIdx.x * 64 + threadIdx.x;
    if (x >= a.w) return;
    const uint64_t o = region(a, blockIdx.y) + x;
    if constexpr (IRREV)
        inv97_line(reinterpret_cast<const float*>(src) + o, a.stride, reinterpret_cast<float*>(dst) + o, a.stride,
                   (int)a.h, (int)a.py);
    else
        inv53_line(src + o, a.stride, dst + o, a.stride, (int)a.h, (int)a.py, true);
}
__global__ __launch_bounds__(256) void k_any_copy(const int32_t* src, int32_t* dst, AnyLevel a) {
    const uint32_t x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.z * 4 + (threadIdx.x >> 6);
    if (x >= a.w || y >= a.h) return;
    const uint64_t o = region(a, blockIdx.y) + (uint64_t)y * a.stride + x;
    dst[o] = src[o];
}
}  // namespace

#include "gk_launch.h"
// One level of tile class (w x h input, parities px / py): forward reads the level's input
// region of `in` and leaves the Mallat output in `out`; inverse the other way round.  `in` /
// `out` are component 0's planes (components cstride apart, grid.y = components x tiles).
void gk_launch_dwt_any(hipStream_t st, bool irrev, bool forward, int32_t* in, int32_t* out, uint32_t stride, uint32_t w,
                       uint32_t h, uint32_t px, uint32_t py, GkTiles tb, GkComps cs, bool partial) {
    if (!w || !h || !tb.count() || !cs.n) return;
    // grid.y = components x tiles (at most 65535: larger sets go one component at a time)
    const uint32_t ng = tb.count() * cs.n <= 65535u ? cs.n : 1u;
    for (uint32_t c = 0; c < cs.n; c += ng) {
        const AnyLevel a{w, h, px, py, partial ? 1u : 0u, tb, cs.cstride, stride};
        const uint32_t nz = tb.count() * ng;
        int32_t* i2 = in + (uint64_t)c * cs.cstride;
        int32_t* o2 = out + (uint64_t)c * cs.cstride;
        const dim3 gw((w + 63) / 64, nz), gh((h + 63) / 64, nz), gc((w + 63) / 64, nz, (h + 3) / 4);
        if (forward) {
            if (irrev) {
                hipLaunchKernelGGL(k_any_fwd_cols<true>, gw, dim3(64), 0, st, i2, o2, a);
                hipLaunchKernelGGL(k_any_fwd_rows<true>, gh, dim3(64), 0, st, i2, o2, a);
            } else {
                hipLaunchKernelGGL(k_any_fwd_cols<false>, gw, dim3(64), 0, st, i2, o2, a);
                hipLaunchKernelGGL(k_any_fwd_rows<false>, gh, dim3(64), 0, st, i2, o2, a);
            }
        } else {
            // rows: Mallat input (in) -> level-below region (out); columns: out -> in
            if (irrev) {
                hipLaunchKernelGGL(k_any_inv_rows<true>, gh, dim3(64), 0, st, i2, o2, a);
                hipLaunchKernelGGL(k_any_inv_cols<true>, gw, dim3(64), 0, st, o2, i2, a);
            } else {
                hipLaunchKernelGGL(k_any_inv_rows<false>, gh, dim3(64), 0, st, i2, o2, a);
                hipLaunchKernelGGL(k_any_inv_cols<false>, gw, dim3(64), 0, st, o2, i2, a);
            }
        }
        hipLaunchKernelGGL(k_any_copy, gc, dim3(256), 0, st, i2, o2, a);   // the result lands in `in`: to `out`
    }
}
