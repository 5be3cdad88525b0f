// gk_xcd.h — XCD-aware workgroup order for the tiled DWT kernels (gfx950: 8 XCDs, one L2 each).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// XCD-aware tile order.  The dispatcher deals workgroups to the 8 XCDs round robin (linear id
// mod 8), so row-major neighbours - which read each other's halo lines - land on different
// XCDs, each with its own L2, and every halo line is fetched from HBM again (C2 level 1 read
// 1.5x its input).  Remapped, XCD k takes the k-th contiguous run of tiles (row-major over x, y,
// z), in order, so a tile's left and upper neighbours were just read through the same L2.
__device__ __forceinline__ uint3 xcd_tile() {
    const uint32_t gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
    const uint32_t lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const uint32_t q = n / 8, r = n % 8, k = lin % 8, j = lin / 8;
    const uint32_t t = k < r ? k * (q + 1) + j : r * (q + 1) + (k - r) * q + j;
    return make_uint3(t % gx, (t / gx) % gy, t / (gx * gy));
}

