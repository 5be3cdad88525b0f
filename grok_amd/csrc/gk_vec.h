// gk_vec.h — four consecutive caller samples as one vector access (16 B int32, 4 B u8 / s8,
// 8 B u16 / s16), widened to int4, and back.  Used by the sample stages and the fused level-1
// DWT kernels when the host found the planes aligned (gk_vec_ok).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gk_common.h"

static __device__ __forceinline__ int4 ld4(const int32_t* p) { return *(const int4*)p; }
static __device__ __forceinline__ int4 ld4(const uint8_t* p) { const uchar4 v = *(const uchar4*)p; return make_int4(v.x, v.y, v.z, v.w); }
static __device__ __forceinline__ int4 ld4(const int8_t* p) { const char4 v = *(const char4*)p; return make_int4(v.x, v.y, v.z, v.w); }
static __device__ __forceinline__ int4 ld4(const uint16_t* p) { const ushort4 v = *(const ushort4*)p; return make_int4(v.x, v.y, v.z, v.w); }
static __device__ __forceinline__ int4 ld4(const int16_t* p) { const short4 v = *(const short4*)p; return make_int4(v.x, v.y, v.z, v.w); }
static __device__ __forceinline__ void st4(int32_t* p, int4 v) { *(int4*)p = v; }
static __device__ __forceinline__ void st4(uint8_t* p, int4 v) { *(uchar4*)p = make_uchar4(v.x, v.y, v.z, v.w); }
static __device__ __forceinline__ void st4(int8_t* p, int4 v) { *(char4*)p = make_char4(v.x, v.y, v.z, v.w); }
static __device__ __forceinline__ void st4(uint16_t* p, int4 v) { *(ushort4*)p = make_ushort4(v.x, v.y, v.z, v.w); }
static __device__ __forceinline__ void st4(int16_t* p, int4 v) { *(short4*)p = make_short4(v.x, v.y, v.z, v.w); }
// four samples from p (vector when v, else one by one: an unaligned plane)
template <class T> static __device__ __forceinline__ int4 ld4v(const T* p, bool v) {
    if (v) return ld4(p);
    return make_int4((int32_t)p[0], (int32_t)p[1], (int32_t)p[2], (int32_t)p[3]);
}
// a plane row pointer p of element type T is aligned for ld4 / st4
template <class T> static __device__ __forceinline__ bool al4(const T* p) { return ((uintptr_t)p % (4 * sizeof(T))) == 0; }
// host: the planes of a fused level-1 kernel take four-sample vector accesses (every plane
// aligned to four samples of es bytes, the row stride a multiple of four samples)
static inline int gk_vec_ok(uint32_t es, const GkPtr3& pl, int nc, uint32_t stride) {
    for (int k = 0; k < nc; ++k)
        if ((uintptr_t)pl.p[k] % (4 * es)) return 0;
    return (stride & 3) == 0;
}
